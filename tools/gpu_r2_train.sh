#!/bin/bash
# Training-parity GPU tests (head + feature extractor backward), then the full GPU suite.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -v -s --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/pytest_train.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_train.log
exit $rc
