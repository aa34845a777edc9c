#!/bin/bash
# Round 4 I: matrix-core BN training parity after the fp64 per-entry statistics
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -rfs \
  -k "batch_stats or train_mode or fe_train or whole_model or sa_backward" > gpurun_out/r4i_train.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/train_step_bench.py --train-fe --bn-train --steps 6 --warmup 2 > gpurun_out/r4i_train_bench.log 2>&1
