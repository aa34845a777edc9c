#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python tools/train_step_bench.py --train-fe --steps 6 --warmup 2 > gpurun_out/train_fe.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_step_bench.py --prefetch 3 > gpurun_out/train_head_p3.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_train_fe" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/train_step_bench.py" --train-fe --steps 4 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_train_fe.log" 2>&1
