#!/bin/bash
# FPS lab A/B (select vs batched, CPU-checked), then FPS/e2e GPU tests, then the bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_lab_sel.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 4096 3000 >> $L 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rfs -k "${1:-fps or e2e}" \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --stage-report --cpu-pairs 1 > gpurun_out/bench1.log 2>&1
echo "BENCH_EXIT $?" >> gpurun_out/bench1.log
