#!/bin/bash
# Round 4 K: kNN grouped tile prefetch A/B (K1 = one position at a time, K2, K4), then kNN parity on K4.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
VARIANTS="K1 K2 K4" bash tools/gpu_ab_micro.sh r4k_ab || exit $?
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/cur.so && cp $L/libdvcp_hip_K4.so $L/libdvcp_hip.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs -k "knn or c3_pair_vs_oracle[0] or c3_pair_vs_oracle[5]" > gpurun_out/r4k_pytest.log 2>&1
rc=$?
cp /tmp/cur.so $L/libdvcp_hip.so
exit $rc
