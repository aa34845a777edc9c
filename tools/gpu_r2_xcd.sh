#!/bin/bash
# Selected GPU tests (pytest -k expression), the C3 bench with the stage report, then the PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE) at one batch in flight.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs -k "$1" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --stage-report > gpurun_out/bench1.log 2>&1 || exit $?
bash tools/gpu_pmc.sh "pmc_$2"
