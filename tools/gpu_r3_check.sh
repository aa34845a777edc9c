#!/bin/bash
# Round-3 check: the rocprofv3 counter list, every GPU test (no -x: see all failures), a short bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-r3a}
(cd /tmp && export TMPDIR=/tmp && timeout -k 5 60 rocprofv3 -L > "$GRAFT_REPO_ROOT/gpurun_out/${tag}_counters.txt" 2>&1)
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -rfs \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stage-report > gpurun_out/${tag}_bench.log 2>&1
