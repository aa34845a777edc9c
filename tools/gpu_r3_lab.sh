#!/bin/bash
# FPS lab (select 512 vs 1024 threads) + a PMC compute pass over the kNN micro-benchmark.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-lab}
L=gpurun_out/fps_lab_$tag.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAVES \
  --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${tag}_knnpmc" -o run -- python3 "$GRAFT_REPO_ROOT/tools/knn_bench.py" \
  > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_knnpmc.log" 2>&1
