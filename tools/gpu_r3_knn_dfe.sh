#!/bin/bash
# kNN parity tests + C3 micro-benchmark, target-feature gradient tests, and the batch-statistics
# train step (per-entry-point times).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3g}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -m gpu -v --timeout 200 \
  --timeout-method thread -rfs -k "knn or bit_identical or feature_grad or dfe_tgt" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/knn_bench.py > gpurun_out/${tag}_knn_bench.log 2>&1 || exit $?
timeout -k 10 300 python tools/train_step_bench.py --train-fe --bn-train --steps 4 --warmup 2 \
  > gpurun_out/${tag}_train_bn.json 2> gpurun_out/${tag}_train_bn.err
