#!/bin/bash
# FPS lab + every GPU test + the C3 bench (no CPU baseline).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-fps}
L=gpurun_out/fps_lab_$tag.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -rfs \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/${tag}_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stage-report > gpurun_out/${tag}_bench.log 2>&1
