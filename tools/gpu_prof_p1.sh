#!/bin/bash
# rocprofv3 kernel stats of the bench at one batch in flight (kernels close to isolated).
TAG=${1:-p1}; shift
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 8 --warmup 2 "$@" > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
echo "PROF_EXIT $?" >> "$ROOT/gpurun_out/prof_$TAG.log"
