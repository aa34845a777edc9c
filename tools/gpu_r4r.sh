#!/bin/bash
# Round 4 R: A/B of S3 (sa1 on the matrix cores, 16-row half tiles for sa2, the per-point pass on
# the matrix cores, FPS floor decay 0.9,
# CPG G3) against P0 (the r4j tree's SA / FPS): tools/sa_bench.py and tools/fps_bench.py; CPG A/B
# G0 (committed) against G3 by tools/knn_bench.py --fast; CPG phase clocks (GD3); then SA / CPG /
# FPS / end-to-end parity on S3.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/cur.so
restore() { cp /tmp/cur.so $L/libdvcp_hip.so; }
for i in 1 2; do
  for v in P0 S3; do
    cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so
    echo "== $v run $i" >> gpurun_out/r4r_sa_ab.log
    DVCP_SKIP_ABI=1 timeout -k 10 200 python tools/sa_bench.py >> gpurun_out/r4r_sa_ab.log 2>&1 || { restore; exit 1; }
    echo "== $v run $i" >> gpurun_out/r4r_fps_ab.log
    DVCP_SKIP_ABI=1 timeout -k 10 200 python tools/fps_bench.py >> gpurun_out/r4r_fps_ab.log 2>&1 || { restore; exit 1; }
  done
done
restore
VARIANTS="G0 G3" bash tools/gpu_ab_micro.sh r4r_cpg_ab || exit $?
timeout -k 10 120 python tools/cpg_diag.py --lib $L/libdvcp_hip_GD3.so > gpurun_out/r4r_cpg_diag.log 2>&1 || exit $?
cp $L/libdvcp_hip_S3.so $L/libdvcp_hip.so
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfs \
  -k "set_abstraction or sa_ or fe_ or fps or c1 or c2_pair_vs_oracle or c3_pair_vs_oracle or cpg or c5 or smoke" \
  > gpurun_out/r4r_pytest.log 2>&1
rc=$?
restore
exit $rc
