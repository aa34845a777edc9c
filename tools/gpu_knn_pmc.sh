#!/bin/bash
# kNN micro-benchmark under one PMC pass: wave cycles vs waiting vs VALU / SMEM issue.
TAG=${1:-knnpmc}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv \
  -d "$ROOT/gpurun_out/${TAG}" -o run -- python3 "$ROOT/tools/knn_bench.py" > "$ROOT/gpurun_out/${TAG}.log" 2>&1
