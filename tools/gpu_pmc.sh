#!/bin/bash
# HBM traffic per kernel launch from PMC counters (MI355X_MICROARCH.md, HBM/rocprofv3): one pass per
# counter block request (FETCH_SIZE and WRITE_SIZE do not fit one pass), bench at one batch in flight.
TAG=${1:-pmc}
ROOT="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d "$ROOT/gpurun_out/${TAG}_$C" -o run \
    -- python3 "$ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 > "$ROOT/gpurun_out/${TAG}_$C.log" 2>&1 || exit $?
done
