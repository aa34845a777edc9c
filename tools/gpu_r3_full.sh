#!/bin/bash
# Every GPU test (no -x: see all failures), then the C3 bench alternating dvcp/libdvcp_hip_A.so (A)
# and the in-tree library (B), twice.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-full}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}_bench.log
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/${tag}_bench.log 2>&1 || exit $?
  done
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
