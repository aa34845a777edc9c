#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_lab_sel.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
