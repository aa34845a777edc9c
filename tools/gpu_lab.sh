#!/bin/bash
# FPS lab variants, then GPU tests + bench + profile (tools/gpu_all.sh).
TAG=${1:-lab}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > gpurun_out/fps_lab_$TAG.log 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 1024 10000 >> gpurun_out/fps_lab_$TAG.log 2>&1 || exit $?
[ "${2:-}" = "all" ] && bash tools/gpu_all.sh "$TAG"
exit 0
