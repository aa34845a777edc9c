#!/bin/bash
# Throughput vs batches in flight and hardware queues (C3, no CPU baseline), alternating configs.
# Usage: [STEPS=48 WARMUP=8] tools/gpu_inflight_sweep.sh "<inflight> <queues>" ...   (default list below)
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("8 16" "8 24" "8 32" "10 20" "10 30" "12 32" "6 24")
for rep in 1 2 3; do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    v=$(timeout -k 10 200 python bench.py --no-cpu-baseline --inflight $1 --hw-queues $2 --steps ${STEPS:-48} --warmup ${WARMUP:-8} 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit $?
    echo "inflight $1 queues $2 rep $rep: $v"
  done
done
