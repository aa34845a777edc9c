#!/bin/bash
# Ball-query parity tests on the in-tree library, the micro-benchmark A (dvcp/libdvcp_hip_A.so)
# against the in-tree library, and per-wave durations from dvcp/libdvcp_hip_D3.so.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-bq}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_paper.py tests/test_gpu_e2e.py -m gpu -q \
  --timeout 200 --timeout-method thread -rfs -k "ball or group or set_abstraction or c3" > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}_bench.log
    timeout -k 10 120 python tools/bq_bench.py 2>&1 | grep -E "^sa" >> gpurun_out/${tag}_bench.log || exit $?
  done
done
cp $L/libdvcp_hip_D3.so $L/libdvcp_hip.so
timeout -k 10 120 python tools/bq_diag.py dur 2>&1 | grep -E "^dur" >> gpurun_out/${tag}_diag.log
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
