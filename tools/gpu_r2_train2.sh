#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/pytest_train.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_train.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/train_step_bench.py --train-fe --steps 6 --warmup 2 > gpurun_out/train_fe.log 2>&1
