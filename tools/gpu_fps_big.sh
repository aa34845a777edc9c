#!/bin/bash
# Split select at C5 size (65536 -> 10000, 4 clouds) and the C3 sizes; roles by ticket (1) / blockIdx (0).
TAG=${1:-big}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_big_$TAG.log
: > $L
timeout -k 10 200 ./tools/fps_lab/fps_lab 4 65536 10000 8 0 1 >> $L 2>&1 || exit $?
timeout -k 10 200 ./tools/fps_lab/fps_lab 4 65536 10000 8 0 0 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 8 10000 10000 8 0 1 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 8 16384 10000 8 0 1 >> $L 2>&1 || exit $?
