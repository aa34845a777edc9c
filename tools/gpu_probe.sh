#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python tools/fps_probe.py > gpurun_out/fps_probe.log 2>&1 &&
DVCP_FPS_NOPRUNE=1 timeout -k 10 300 python tools/fps_probe.py >> gpurun_out/fps_probe.log 2>&1 &&
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q --timeout 300 -rfs -k "knn or fps" > gpurun_out/pytest_knn.log 2>&1
echo "EXIT $?" >> gpurun_out/pytest_knn.log
