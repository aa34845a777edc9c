#!/bin/bash
# kNN round-5 check: A/B of two library builds on the C3 kNN micro-benchmark, PMC HBM bytes of each
# (FETCH_SIZE and WRITE_SIZE in separate passes), then the kNN / BN-training / one C3 e2e tests.
# Usage: VARIANTS="k0 k1" tools/gpu_knn_r5.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
ROOT=$PWD
tag=${1:-knn}
L=$ROOT/deepvcp-pointcloud-registration_amd/dvcp
bash tools/gpu_ab_micro.sh ${tag}_ab || exit 1
for v in $VARIANTS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && DVCP_LIB_PATH=$L/libdvcp_hip_$v.so timeout -s KILL 120 rocprofv3 --pmc $c \
      --output-format csv -d "$ROOT/gpurun_out/${tag}_pmc_${v}_$c" -o run -- python3 "$ROOT/tools/knn_bench.py" --fast \
      > "$ROOT/gpurun_out/${tag}_pmc_${v}_$c.log" 2>&1) || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_train.py tests/test_gpu_e2e.py -k "knn or many_centres or c3_pair_vs_oracle and 0" \
  > gpurun_out/${tag}_pytest.log 2>&1
