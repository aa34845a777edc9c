#!/bin/bash
# FPS lab A/B of the split select: fps_lab_head (the committed kernel) against fps_lab (the tree),
# then the FPS GPU tests.
TAG=${1:-ab2}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_ab2_$TAG.log
: > $L
for r in 1 2; do
for lab in fps_lab_head fps_lab; do
  echo "== $lab run $r" >> $L
  timeout -k 10 120 ./tools/fps_lab/$lab 8 10000 10000 8 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 8 16384 10000 8 >> $L 2>&1 || exit $?
  timeout -k 10 200 ./tools/fps_lab/$lab 4 65536 10000 8 >> $L 2>&1 || exit $?
done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "fps or split" --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_fps_$TAG.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_fps_$TAG.log
