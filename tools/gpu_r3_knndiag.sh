#!/bin/bash
# kNN per-wave diagnostics (dvcp/libdvcp_hip_D.so, a DVCP_KNN_DIAG build) and the kNN bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-knndiag}
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 120 python tools/knn_bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit $?
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_main.so
cp $L/libdvcp_hip_D.so $L/libdvcp_hip.so
timeout -k 10 120 python tools/knn_diag.py > gpurun_out/${tag}.log 2>&1
rc=$?
cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so
exit $rc
