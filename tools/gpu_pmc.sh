#!/bin/bash
# PMC passes over the C3 bench at one batch in flight (MI355X_MICROARCH.md, HBM / rocprofv3 PMC
# slots): FETCH_SIZE and WRITE_SIZE each need a pass of their own (TCC slots); the compute pass
# takes rocprofv3's derived MfmaUtil / VALUBusy / VALUUtilization and raw SQ instruction counts
# (8 SQ counters + GRBM_GUI_ACTIVE).  Then tools/pmc_summary.py -> gpurun_out/<tag>_pmc_summary.json.
# CONFIG=c5: the same passes over the C5 bench (bench.py --config c5).
TAG=${1:-pmc}
CFG=${CONFIG:-c3}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/${TAG}_$name" -o run \
    -- python3 "$ROOT/bench.py" --config "$CFG" --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 --iso-steps 1 \
    > "$ROOT/gpurun_out/${TAG}_$name.log" 2>&1
}
run FETCH FETCH_SIZE || exit $?
run WRITE WRITE_SIZE || exit $?
run COMPUTE MfmaUtil VALUBusy VALUUtilization SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES SQ_WAVES || exit $?
python3 "$ROOT/tools/pmc_summary.py" "$ROOT/gpurun_out/${TAG}_FETCH" "$ROOT/gpurun_out/${TAG}_WRITE" \
  "$ROOT/gpurun_out/${TAG}_COMPUTE" > "$ROOT/gpurun_out/${TAG}_pmc_summary.json"
