#!/bin/bash
# Training-step A/B of library builds (frozen-BN extractor training, tools/train_step_bench.py --train-fe):
# the in-tree library against dvcp/libdvcp_hip_<V>.so, alternating, 2 rounds.
# Usage: V=name tools/gpu_train_ab.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-tab}
L=$PWD/deepvcp-pointcloud-registration_amd/dvcp
for i in 1 2; do
  echo "== in-tree run $i" >> gpurun_out/${tag}.log
  timeout -k 10 200 python tools/train_step_bench.py --train-fe >> gpurun_out/${tag}.log 2>&1 || exit 1
  echo "== $V run $i" >> gpurun_out/${tag}.log
  DVCP_LIB_PATH=$L/libdvcp_hip_$V.so timeout -k 10 200 python tools/train_step_bench.py --train-fe \
    >> gpurun_out/${tag}.log 2>&1 || exit 1
done
