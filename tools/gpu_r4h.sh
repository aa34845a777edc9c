#!/bin/bash
# Round 4 H: matrix-core batch-statistics BN for all three tables -- training parity, the training
# step bench and its per-kernel profile.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -rfs \
  -k "batch_stats or train_mode or fe_train or whole_model or sa_backward" > gpurun_out/r4h_train.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/train_step_bench.py --train-fe --bn-train --steps 6 --warmup 2 > gpurun_out/r4h_train_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r4h_prof_train" -o run \
  -- python3 "$GRAFT_REPO_ROOT/tools/train_step_bench.py" --train-fe --bn-train --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/r4h_prof_train.log" 2>&1
