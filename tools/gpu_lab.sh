#!/bin/bash
# FPS lab configurations; with "all": GPU tests + bench + profile (tools/gpu_all.sh).
TAG=${1:-lab}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_lab_$TAG.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 1024 10000 >> $L 2>&1 || exit $?
if [ "${2:-}" = "all" ]; then bash tools/gpu_all.sh "$TAG"; fi
exit 0
