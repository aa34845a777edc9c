#!/bin/bash
# SA / kNN parity tests on the in-tree library (B), then tools/sa_bench.py alternating
# dvcp/libdvcp_hip_A.so (A) and B, and tools/knn_bench.py on B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-absa}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_configs.py -m gpu -q \
  --timeout 200 --timeout-method thread -rfs -k "set_abstraction or sa_mlp or knn or c3 or c2" > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 120 python tools/knn_bench.py 2>&1 | grep -E "^knn" > gpurun_out/${tag}_knn.log || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}.log
    timeout -k 10 120 python tools/sa_bench.py 2>&1 | grep -E "^sa" >> gpurun_out/${tag}.log || exit $?
  done
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
