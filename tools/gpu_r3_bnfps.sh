#!/bin/bash
# FPS lab (select timings) + FPS tests, batch-statistics train tests + train step bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3k}
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -m gpu -v --timeout 240 \
  --timeout-method thread -rfs -k "batch_stats or train_mode or direct_module or feature_grad or bit_identical or fps" \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/train_step_bench.py --train-fe --bn-train --steps 4 --warmup 2 \
  > gpurun_out/${tag}_train_bn.json 2> gpurun_out/${tag}_train_bn.err
