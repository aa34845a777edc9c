#!/bin/bash
# A/B of library builds with the full C3 bench (no CPU baseline): dvcp/libdvcp_hip_<V>.so for V in
# $VARIANTS, alternating, $ROUNDS rounds (default 2).  Each variant is loaded through DVCP_LIB_PATH;
# the in-tree library is never touched.
# Usage: VARIANTS="X Y" tools/gpu_ab_lib.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-ab}
L=$PWD/deepvcp-pointcloud-registration_amd/dvcp
for i in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    echo "== $v run $i" >> gpurun_out/${tag}.log
    DVCP_LIB_PATH=$L/libdvcp_hip_$v.so timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline \
      >> gpurun_out/${tag}.log 2>&1 || exit 1
  done
done
