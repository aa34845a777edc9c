#!/bin/bash
# Selected GPU tests by -k expression (arg 1), verbose with prints.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -rfs -k "$1" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
exit $rc
