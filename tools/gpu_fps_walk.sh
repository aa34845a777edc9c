#!/bin/bash
# fps_lab at the FE's FPS shapes (select vs walk variants).
set -e
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for args in "16 16384 10000" "16 10000 10000" "4 8192 4096"; do
  echo "== $args"
  timeout -k 10 120 tools/fps_lab/fps_lab $args
done
