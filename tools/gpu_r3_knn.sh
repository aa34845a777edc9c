#!/bin/bash
# kNN parity tests + C3 micro-benchmark.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3k}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -m gpu -v --timeout 200 \
  --timeout-method thread -rfs -k "knn" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/knn_bench.py > gpurun_out/${tag}_knn_bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1
