#!/bin/bash
# FPS lab counters (rounds, scans, rescans per reason, per-wave phase clocks) at the C3 sizes, then
# the C5 bench (N = 65536, K = 256, fp16 features).  Build the lab first on the CPU:
# make -C tools/fps_lab fps_lab.  Usage: tools/gpu_fps_c5.sh <tag>
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-fc}
timeout -k 10 240 ./tools/fps_lab/fps_lab 16 16384 10000 > gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
timeout -k 10 120 ./tools/fps_lab/fps_lab 16 10000 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
# a variant lab binary, when one was built (e.g. -DDVCP_FPS_UPD_PF=1 -o fps_lab_pf)
for v in tools/fps_lab/fps_lab_*; do
  [ -x "$v" ] || continue
  echo "== $v" >> gpurun_out/${tag}_fps_lab.log
  timeout -k 10 240 "$v" 16 16384 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
  timeout -k 10 120 "$v" 16 10000 10000 >> gpurun_out/${tag}_fps_lab.log 2>&1 || exit $?
done
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline > gpurun_out/${tag}_bench_c5.log 2>&1
