#!/bin/bash
# C3 bench (default settings, no CPU baseline) and the rocprofv3 kernel stats of one batch in
# flight (isolated per-kernel durations).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3q}
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_iso" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --inflight 1 --no-cpu-baseline > "$ROOT/gpurun_out/${tag}_iso.log" 2>&1
