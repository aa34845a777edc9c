#!/bin/bash
# rocprofv3 kernel statistics of the batch-statistics training step and of the C5 forward (one batch
# in flight).  Usage: tools/gpu_prof_extra.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-px}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_train_bn" -o run \
  -- python3 "$ROOT/tools/train_step_bench.py" --train-fe --bn-train --steps 4 > "$ROOT/gpurun_out/${tag}_train_bn.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_c5_iso" -o run \
  -- python3 "$ROOT/bench.py" --config c5 --no-cpu-baseline --inflight 1 --steps 4 --warmup 2 > "$ROOT/gpurun_out/${tag}_c5_iso.log" 2>&1
