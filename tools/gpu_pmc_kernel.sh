#!/bin/bash
# One PMC pass (counters given as arguments) over the bench at one batch in flight; also lists the
# available counters once.  Usage: bash tools/gpu_pmc_kernel.sh <tag> <counter> [<counter> ...]
TAG=$1; shift
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
[ -f "$ROOT/gpurun_out/avail.txt" ] || timeout -s KILL 60 rocprofv3 --list-avail > "$ROOT/gpurun_out/avail.txt" 2>&1
timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/$TAG" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 3 --warmup 1 > "$ROOT/gpurun_out/$TAG.log" 2>&1
