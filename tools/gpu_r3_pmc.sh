#!/bin/bash
# The batch-statistics train test (B = 1, 2) and the PMC passes.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 240 --timeout-method thread -rfs \
  -k "whole_model_train_mode or direct_module" > gpurun_out/${tag}_pytest_train.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/${tag}_pytest_train.log
bash tools/gpu_pmc.sh ${tag}
