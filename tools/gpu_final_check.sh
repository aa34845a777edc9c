#!/bin/bash
# Every GPU test and smoke on the tree as committed, then the C5 bench.  Usage: tools/gpu_final_check.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-fin}
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > gpurun_out/${tag}_bench_c5.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench.log 2>&1
