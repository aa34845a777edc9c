#!/bin/bash
# One PMC pass over the head-training bench (counters as arguments).  Usage: bash tools/gpu_pmc_train.sh <tag> <counters...>
TAG=$1; shift
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/$TAG" -o run \
  -- python3 "$ROOT/tools/train_step_bench.py" --steps 3 --warmup 1 > "$ROOT/gpurun_out/$TAG.log" 2>&1
