#!/bin/bash
# bench at 1, 2, 3 and 4 batches in flight (no CPU baseline)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for P in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 8 --warmup 2 --inflight $P --no-cpu-baseline > gpurun_out/bench_inflight_$P.log 2>&1 || exit $?
done
