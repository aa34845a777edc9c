#!/bin/bash
# kNN: every kNN parity test, then the C3-shape A/B micro-benchmark (tools/knn_bench.py).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-knn}
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -v --timeout 200 --timeout-method thread -rfs \
  -k "knn" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/knn_bench.py > gpurun_out/${tag}_bench.log 2>&1
