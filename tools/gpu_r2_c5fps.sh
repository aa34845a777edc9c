#!/bin/bash
# Split-FPS change check: FPS / C5 GPU tests, then the C5 bench line.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs -k "fps or c5 or C5" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config c5 --steps 8 --warmup 2 --stage-report > gpurun_out/bench_c5.log 2>&1
