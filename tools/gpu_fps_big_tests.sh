#!/bin/bash
# Split select above 16384 points: lab at C5 size + the FPS / config / e2e GPU tests.
TAG=${1:-bt}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_big_$TAG.log
: > $L
timeout -k 10 200 ./tools/fps_lab/fps_lab 4 65536 10000 8 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -k "fps or e2e or c5 or split" --timeout 400 \
  --timeout-method thread > gpurun_out/pytest_big_$TAG.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_big_$TAG.log
