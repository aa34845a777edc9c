#!/bin/bash
# GPU parity tests, then bench + rocprofv3 (tools/bench_and_profile.sh) if no test crashed.
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q --timeout 400 -rfs > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_gpu_$TAG.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  bash tools/bench_and_profile.sh "$TAG"
fi
