#!/bin/bash
# FPS second certification pass: lab A/B (fps_lab = DVCP_FPS_RECERT 1, fps_lab_r0 = 0; one workgroup
# per cloud and the split select at S = 4 / 8) + the FPS / end-to-end GPU tests.
TAG=${1:-rc}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_recert_$TAG.log
: > $L
for lab in fps_lab_r0 fps_lab; do
  echo "== $lab" >> $L
  timeout -k 10 200 ./tools/fps_lab/$lab 16 16384 10000 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 16 10000 10000 >> $L 2>&1 || exit $?
  timeout -k 10 60 ./tools/fps_lab/$lab 16 2500 1250 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 8 10000 10000 4 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 8 10000 10000 8 >> $L 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "fps or e2e" --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_fps_$TAG.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_fps_$TAG.log
