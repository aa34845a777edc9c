#!/bin/bash
# Ball-query count outputs of the in-tree library and of diagnostic builds dvcp/libdvcp_hip_D*.so.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-bqdump}
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_main.so
for v in main $(cd $L && ls libdvcp_hip_D*.so 2>/dev/null | sed 's/libdvcp_hip_//; s/.so//'); do
  if [ $v = main ]; then cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so; else cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so; fi
  timeout -k 10 120 python tools/bq_dump.py ${tag}_$v > gpurun_out/${tag}_$v.log 2>&1 || break
done
cp /tmp/libdvcp_hip_main.so $L/libdvcp_hip.so
