#!/bin/bash
# Round evidence in one GPU call: GPU parity tests, bench (with CPU baseline) + rocprofv3 kernel
# stats of the same command (tools/bench_and_profile.sh), then the PMC HBM-traffic passes.
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/bench_and_profile.sh "$TAG" || exit $?
cd "$GRAFT_REPO_ROOT" && bash tools/gpu_pmc.sh "pmc_$TAG"
