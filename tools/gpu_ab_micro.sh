#!/bin/bash
# A/B of library builds with the C3-shape kNN + target-DFE + CPG micro-benchmark (tools/knn_bench.py
# --fast): the variants dvcp/libdvcp_hip_<V>.so for V in $VARIANTS (default: every such file),
# alternating, two rounds; the in-tree library is restored afterwards.
# Usage: VARIANTS="K1 K4" tools/gpu_ab_micro.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-abm}
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_cur.so
vs=${VARIANTS:-$(ls $L | sed -n 's/^libdvcp_hip_\(.*\)\.so$/\1/p' | tr '\n' ' ')}
for i in 1 2; do
  for v in $vs; do
    cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so
    echo "== $v run $i" >> gpurun_out/${tag}.log
    DVCP_SKIP_ABI=1 timeout -k 10 200 python tools/knn_bench.py --fast >> gpurun_out/${tag}.log 2>&1 || { cp /tmp/libdvcp_hip_cur.so $L/libdvcp_hip.so; exit 1; }
  done
done
cp /tmp/libdvcp_hip_cur.so $L/libdvcp_hip.so
