#!/bin/bash
# FPS lab (N=16384 / 10000 / 1024) + the FPS and end-to-end GPU tests.
TAG=${1:-q}
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=gpurun_out/fps_lab_$TAG.log
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> $L 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 1024 10000 >> $L 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests -m gpu -q -k "fps or e2e or sa" --timeout 400 > gpurun_out/pytest_fps_$TAG.log 2>&1
echo "PYTEST_EXIT $?" >> gpurun_out/pytest_fps_$TAG.log
