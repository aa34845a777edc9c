#!/bin/bash
# Selected GPU tests (-k "$2") on the in-tree library (B), the FPS lab, then the C3 bench
# alternating dvcp/libdvcp_hip_A.so (A) and B, twice.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-fpsab}
sel=${2:-"fps or c3 or c2 or paper or split"}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -rfs -k "$sel" \
  > gpurun_out/${tag}_pytest.log 2>&1 || exit $?
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}_bench.log
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/${tag}_bench.log 2>&1 || exit $?
  done
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
