#!/bin/bash
# Quick GPU iteration: selected GPU tests (pytest -k EXPR), then a bench without the CPU baseline.
# Usage: bash tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args...]
TAG=$1; K=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/q_pytest_$TAG.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/q_pytest_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --stage-report "$@" > gpurun_out/q_bench_$TAG.log 2>&1
rc=$?
echo "BENCH_EXIT $rc" >> gpurun_out/q_bench_$TAG.log
exit $rc
