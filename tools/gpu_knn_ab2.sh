#!/bin/bash
# kNN variants: micro A/B, then WRITE_SIZE / FETCH_SIZE of each (one PMC pass per counter).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ROOT=$PWD; tag=${1:-knn2}
L=$ROOT/deepvcp-pointcloud-registration_amd/dvcp
bash tools/gpu_ab_micro.sh ${tag}_ab || exit 1
for v in $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && DVCP_LIB_PATH=$L/libdvcp_hip_$v.so timeout -s KILL 120 rocprofv3 --pmc $c \
      --output-format csv -d "$ROOT/gpurun_out/${tag}_pmc_${v}_$c" -o run -- python3 "$ROOT/tools/knn_bench.py" --fast \
      > "$ROOT/gpurun_out/${tag}_pmc_${v}_$c.log" 2>&1) || exit 1
  done
done
