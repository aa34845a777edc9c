#!/bin/bash
# FPS lab A/B: fps_lab_head (the committed kernel) against fps_lab (the working tree).
TAG=${1:-ab}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_ab_$TAG.log
: > $L
for lab in fps_lab_head fps_lab; do
  echo "== $lab" >> $L
  timeout -k 10 200 ./tools/fps_lab/$lab 16 16384 10000 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 16 10000 10000 >> $L 2>&1 || exit $?
  timeout -k 10 120 ./tools/fps_lab/$lab 8 10000 10000 8 >> $L 2>&1 || exit $?
done
timeout -k 10 200 ./tools/fps_lab/fps_lab 4 65536 10000 8 >> $L 2>&1 || exit $?
