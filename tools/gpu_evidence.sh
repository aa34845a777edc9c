#!/bin/bash
# Round evidence on one GPU box, in two calls (each within gpurun's 20-minute limit):
#   PART=1: every GPU test, smoke, the C3 bench (with the CPU baseline and the per-stage report);
#   PART=2: rocprofv3 kernel statistics with one batch in flight (iso) and at the bench's default
#           lanes (p10), the PMC passes (tools/gpu_pmc.sh) at C3 and C5, the C5 bench and the C3
#           bench with the literal DFE chain (--dfe literal).
# Usage: PART=1 tools/gpu_evidence.sh <tag>; PART=2 tools/gpu_evidence.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-ev}
ROOT="$GRAFT_REPO_ROOT"
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfs \
    > gpurun_out/${tag}_pytest_gpu.log 2>&1
  rc=$?
  echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --stage-report > gpurun_out/${tag}_bench.log 2>&1 || exit $?
  exit 0
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_iso" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 6 --warmup 2 > "$ROOT/gpurun_out/${tag}_iso.log" 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_p10" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$ROOT/gpurun_out/${tag}_p10.log" 2>&1 || exit $?
bash "$ROOT/tools/gpu_pmc.sh" "${tag}" || exit $?
CONFIG=c5 bash "$ROOT/tools/gpu_pmc.sh" "${tag}_c5" || exit $?
cd "$ROOT" && timeout -k 10 200 python bench.py --config c5 > gpurun_out/${tag}_bench_c5.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --dfe literal > gpurun_out/${tag}_bench_dfe_literal.log 2>&1
