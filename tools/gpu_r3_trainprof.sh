#!/bin/bash
# rocprofv3 kernel stats of the whole-model batch-statistics train step.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3f}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_tprof" -o run \
  -- python3 "$ROOT/tools/train_step_bench.py" --train-fe --bn-train --steps 3 --warmup 1 \
  > "$ROOT/gpurun_out/${tag}_tprof.log" 2>&1
