#!/bin/bash
# kNN parity + micro-benchmark on the in-tree library, then the ball-query micro-benchmark on the
# in-tree library and on diagnostic builds dvcp/libdvcp_hip_D*.so (swapped in one at a time).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-diag}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -m gpu -q --timeout 200 \
  --timeout-method thread -rfs -k "knn" > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 120 python tools/knn_bench.py 2>&1 | grep -E "^knn" > gpurun_out/${tag}_knn.log || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_main.so
for v in main $(cd $L && ls libdvcp_hip_D*.so 2>/dev/null | sed 's/libdvcp_hip_//; s/.so//'); do
  if [ $v = main ]; then cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so; else cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so; fi
  echo "== $v" >> gpurun_out/${tag}_bq.log
  timeout -k 10 120 python tools/bq_bench.py 2>&1 | grep -E "^sa" >> gpurun_out/${tag}_bq.log || exit $?
done
cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so
