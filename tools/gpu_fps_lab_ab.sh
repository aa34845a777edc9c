#!/bin/bash
# A/B of the FPS lab against tools/fps_lab/fps_lab_old (the previous commit's kernel), alternating.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
for args in "16 16384 10000" "16 10000 10000"; do
  for rep in 1 2; do
    for bin in fps_lab_old fps_lab; do
      echo "== $bin $args"
      timeout -k 10 120 tools/fps_lab/$bin $args || exit $?
    done
  done
done
