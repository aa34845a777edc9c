#!/bin/bash
# SA parity + split-3 accuracy tests on the in-tree library (B), then tools/sa_bench.py and the C3
# bench alternating dvcp/libdvcp_hip_A.so (A) and B.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-split}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py tests/test_gpu_configs.py -m gpu -v -s \
  --timeout 200 --timeout-method thread -rfs -k "set_abstraction or split3 or row_map or c3 or c2 or sa_ or fps" \
  > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}_sa.log
    timeout -k 10 120 python tools/sa_bench.py 2>&1 | grep -E "^sa" >> gpurun_out/${tag}_sa.log || exit $?
  done
done
for v in A B; do
  if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
  echo "== $v" >> gpurun_out/${tag}_bench.log
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/${tag}_bench.log 2>&1 || exit $?
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
