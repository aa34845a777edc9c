#!/bin/bash
# Selected GPU tests (args: pytest -k expression), then the C3 and C5 bench lines.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs -k "$1" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || exit $?
timeout -k 10 400 python bench.py --config c5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
