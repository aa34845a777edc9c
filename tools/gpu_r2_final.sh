#!/bin/bash
# Round evidence: every GPU test, smoke, the C3 bench (with CPU baseline), the C5 stress bench,
# an isolated rocprofv3 kernel-trace capture, then the PMC traffic passes.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --stage-report > gpurun_out/bench1.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --config c5 --steps 8 --warmup 2 --stage-report > gpurun_out/bench_c5.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_iso" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 6 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_iso.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_p10" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_p10.log" 2>&1 || exit $?
bash "$GRAFT_REPO_ROOT/tools/gpu_pmc.sh" "${1:-pmc_r2v}"
