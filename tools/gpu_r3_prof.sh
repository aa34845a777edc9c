#!/bin/bash
# Paper FP test, the whole-model batch-statistics train step (per-entry-point times), and the
# rocprofv3 kernel stats of a short bench run (per FPS instance).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3e}
ROOT="$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_paper.py tests/test_gpu_train.py -m gpu -v --timeout 120 \
  --timeout-method thread -rfs -k "feature_propagation or bit_identical or feature_grad" \
  > gpurun_out/${tag}_pytest.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/${tag}_pytest.log
timeout -k 10 300 python tools/train_step_bench.py --train-fe --bn-train --steps 6 --warmup 2 \
  > gpurun_out/${tag}_train_bn.json 2> gpurun_out/${tag}_train_bn.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/${tag}_prof" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$ROOT/gpurun_out/${tag}_prof.log" 2>&1
