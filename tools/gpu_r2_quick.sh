#!/bin/bash
# Selected GPU tests (args: pytest -k expression), then the default bench with the stage report.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs -s -k "$1" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 400 python bench.py --stage-report > gpurun_out/bench1.log 2>&1
echo "BENCH_EXIT $?" >> gpurun_out/bench1.log
