#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q --timeout 400 -rfs > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --stage-report > gpurun_out/bench1.log 2>&1
  echo "BENCH_EXIT $?" >> gpurun_out/bench1.log
fi
