#!/bin/bash
# Stall breakdown of every kernel of the C3 step (bench.py, one batch in flight): two PMC passes
# (wave cycles split into waiting / issue-stalled / issuing; instruction mix + LDS bank conflicts),
# summarised per kernel by tools/micro_pmc.py.  Usage: tools/gpu_stall_pmc.sh <tag>
TAG=${1:-stall}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
B="$ROOT/bench.py --no-cpu-baseline --inflight 1 --steps 3 --warmup 1 --iso-steps 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$ROOT/gpurun_out/${TAG}_A" -o run -- python3 $B > "$ROOT/gpurun_out/${TAG}_A.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_MFMA \
  SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
  -d "$ROOT/gpurun_out/${TAG}_B" -o run -- python3 $B > "$ROOT/gpurun_out/${TAG}_B.log" 2>&1 || exit $?
python3 "$ROOT/tools/micro_pmc.py" "$ROOT/gpurun_out/${TAG}_A" "$ROOT/gpurun_out/${TAG}_B" > "$ROOT/gpurun_out/${TAG}_summary.txt"
