#!/bin/bash
# FPS change check: FPS / e2e GPU tests, one-batch bench (FPS launch time) and three 8-lane benches.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fps or e2e" > gpurun_out/fab_pytest.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 > gpurun_out/fab_p1.log 2>&1 || exit $?
for i in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fab_p8_$i.log 2>&1 || exit $?; done
