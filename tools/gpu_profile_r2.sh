#!/bin/bash
# rocprofv3 kernel-trace/stats of the bench at one batch in flight (isolated per-kernel times) and at
# the default 8 batches, then the PMC traffic passes (FETCH_SIZE, WRITE_SIZE; tools/gpu_pmc.sh).
TAG=${1:-r2}
ROOT="$GRAFT_REPO_ROOT"
mkdir -p "$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_${TAG}_iso" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 6 --warmup 2 > "$ROOT/gpurun_out/prof_${TAG}_iso.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_${TAG}_p8" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$ROOT/gpurun_out/prof_${TAG}_p8.log" 2>&1 || exit $?
bash "$ROOT/tools/gpu_pmc.sh" "pmc_${TAG}"
