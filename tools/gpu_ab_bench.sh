#!/bin/bash
# A/B of two prebuilt libraries (tools/ab/libdvcp_hip_{A,B}.so) on the default bench, alternating.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=deepvcp-pointcloud-registration_amd/dvcp/libdvcp_hip.so
for v in A B A B; do
  cp tools/ab/libdvcp_hip_$v.so $L
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 48 > gpurun_out/ab_$v.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log) $(grep -o '"latency_ms_single_batch": [0-9.]*' gpurun_out/ab_$v.log)" >> gpurun_out/ab_summary.log
done
cp tools/ab/libdvcp_hip_A.so $L
