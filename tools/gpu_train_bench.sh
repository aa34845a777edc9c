#!/bin/bash
# Head-training step bench + rocprofv3 kernel stats of the same command.
TAG=${1:-t}
ROOT="$GRAFT_REPO_ROOT"
cd "$ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python tools/train_step_bench.py > gpurun_out/train_bench_$TAG.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_train_$TAG" -o run \
  -- python3 "$ROOT/tools/train_step_bench.py" --steps 5 > "$ROOT/gpurun_out/prof_train_$TAG.log" 2>&1
