#!/bin/bash
# Batch-statistics train tests + the whole-model train step (per-entry-point times) + kernel stats.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3h}
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -m gpu -v --timeout 240 --timeout-method thread -rfs \
  -k "batch_stats or train_mode or direct_module or feature_grad or bit_identical" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/train_step_bench.py --train-fe --bn-train --steps 4 --warmup 2 \
  > gpurun_out/${tag}_train_bn.json 2> gpurun_out/${tag}_train_bn.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_tprof" -o run \
  -- python3 "$ROOT/tools/train_step_bench.py" --train-fe --bn-train --steps 2 --warmup 1 \
  > "$ROOT/gpurun_out/${tag}_tprof.log" 2>&1
