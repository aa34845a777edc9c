#!/bin/bash
# FPS lab: candidate-target sweep (fps_lab_t<T>, DVCP_FPS_SEL_TARGET = T; fps_lab = 64).
TAG=${1:-tg}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_target_$TAG.log
: > $L
for lab in fps_lab_t48 fps_lab fps_lab_t80 fps_lab_t96; do
  echo "== $lab" >> $L
  timeout -k 10 200 ./tools/fps_lab/$lab 16 16384 10000 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 16 10000 10000 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 8 10000 10000 8 >> $L 2>&1 || exit $?
done
