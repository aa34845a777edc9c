#!/bin/bash
# Candidate library dvcp/libdvcp_hip_A.so (A): kNN / C3 / DFE parity tests and the kNN
# micro-benchmark on A, then the C3 bench alternating A and the in-tree library (B).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-knnsl}
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so
cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -rfs -k "knn or c3 or dfe" \
  > gpurun_out/${tag}_pytest.log 2>&1 || { cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; exit 1; }
timeout -k 10 120 python tools/knn_bench.py > gpurun_out/${tag}_knnbench.log 2>&1 || { cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; exit 1; }
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp $L/libdvcp_hip_A.so $L/libdvcp_hip.so; else cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}_bench.log
    timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/${tag}_bench.log 2>&1 || exit $?
  done
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
