#!/bin/bash
# Throughput vs batches in flight (P) and hardware queues (Q), no CPU baseline.
# Usage: bash tools/gpu_sweep.sh "<P list>" "<Q list>" [bench args...]
PS=$1; QS=$2; shift 2
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for Q in $QS; do
  for P in $PS; do
    timeout -k 10 200 python bench.py --steps 32 --warmup 4 --inflight $P --hw-queues $Q --no-cpu-baseline "$@" > gpurun_out/sw_${Q}_${P}.log 2>&1 || exit $?
    echo "Q=$Q P=$P $(grep -o '"value": [0-9.]*' gpurun_out/sw_${Q}_${P}.log) $(grep -o '"latency_ms_single_batch": [0-9.]*' gpurun_out/sw_${Q}_${P}.log)" >> gpurun_out/sweep.log
  done
done
