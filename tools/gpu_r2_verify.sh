#!/bin/bash
# GPU tests (one process, per-test timeouts), smoke, then a short bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --stage-report > gpurun_out/bench1.log 2>&1
echo "BENCH_EXIT $?" >> gpurun_out/bench1.log
