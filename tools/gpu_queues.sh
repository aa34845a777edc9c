#!/bin/bash
# bench throughput vs hardware queues per process and batches in flight (no CPU baseline)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for Q in 4 8 16; do
  for P in 4 6; do
    echo "Q=$Q P=$P" >> gpurun_out/queues.log
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --steps 8 --warmup 2 --inflight $P --no-cpu-baseline > gpurun_out/q_${Q}_${P}.log 2>&1 || exit $?
    grep -o '"value": [0-9.]*' gpurun_out/q_${Q}_${P}.log >> gpurun_out/queues.log
  done
done
