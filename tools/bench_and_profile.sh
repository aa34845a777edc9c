#!/bin/bash
# 1-GPU bench (with the CPU baseline) + rocprofv3 kernel-trace/stats of the same workload.
# Usage: bash tools/bench_and_profile.sh <tag>
TAG=${1:-r1}
ROOT="$GRAFT_REPO_ROOT"
cd "$ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python bench.py --stage-report > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "BENCH_EXIT $rc" >> gpurun_out/bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
echo "PROF_EXIT $?" >> "$ROOT/gpurun_out/prof_$TAG.log"
