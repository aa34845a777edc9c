#!/bin/bash
# CPG parity tests (forward + backward) and the C3-shape micro-benchmark (kNN, DFE, CPG).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3m}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_e2e.py -m gpu -v \
  --timeout 200 --timeout-method thread -rfs -k "cpg or e2e_c1 or head_train" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/knn_bench.py > gpurun_out/${tag}_knn_bench.log 2>&1
