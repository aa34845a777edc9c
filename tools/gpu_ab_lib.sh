#!/bin/bash
# A/B of library builds with the full C3 bench (no CPU baseline): dvcp/libdvcp_hip_<V>.so for V in
# $VARIANTS, alternating, $ROUNDS rounds (default 2); the in-tree library is restored afterwards.
# Usage: VARIANTS="X Y" tools/gpu_ab_lib.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-ab}
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_cur.so
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so
    echo "== $v run $i" >> gpurun_out/${tag}.log
    DVCP_SKIP_ABI=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/${tag}.log 2>&1 \
      || { cp /tmp/libdvcp_hip_cur.so $L/libdvcp_hip.so; exit 1; }
  done
done
cp /tmp/libdvcp_hip_cur.so $L/libdvcp_hip.so
