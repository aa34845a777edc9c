#!/bin/bash
# Per-wave clock stamps of the ball-query kernel from diagnostic builds (dvcp/libdvcp_hip_D3..5.so).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-bqdiag}
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_main.so
for v in 3:dur 4:start 5:end; do
  cp $L/libdvcp_hip_D${v%%:*}.so $L/libdvcp_hip.so
  timeout -k 10 120 python tools/bq_diag.py ${v##*:} 2>&1 | grep -vE "amdgpu.ids" >> gpurun_out/${tag}.log || break
done
cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so
