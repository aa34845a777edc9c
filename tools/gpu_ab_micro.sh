#!/bin/bash
# A/B of library builds with a micro-benchmark (default: the C3-shape kNN + target-DFE + CPG one,
# tools/knn_bench.py --fast; BENCH="tools/sa_bench.py" for the set-abstraction tables): the variants
# dvcp/libdvcp_hip_<V>.so for V in $VARIANTS (default: every such file), alternating, two rounds,
# each loaded through DVCP_LIB_PATH (the in-tree library is never touched).
# Usage: VARIANTS="K1 K4" [BENCH="tools/sa_bench.py"] tools/gpu_ab_micro.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-abm}
L=$PWD/deepvcp-pointcloud-registration_amd/dvcp
vs=${VARIANTS:-$(ls $L | sed -n 's/^libdvcp_hip_\(.*\)\.so$/\1/p' | tr '\n' ' ')}
bench=${BENCH:-tools/knn_bench.py --fast}
for i in 1 2; do
  for v in $vs; do
    echo "== $v run $i" >> gpurun_out/${tag}.log
    DVCP_LIB_PATH=$L/libdvcp_hip_$v.so timeout -k 10 200 python $bench >> gpurun_out/${tag}.log 2>&1 \
      || exit 1
  done
done
