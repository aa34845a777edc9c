#!/bin/bash
# A/B of library builds with the C3-shape kNN + target-DFE + CPG micro-benchmark (tools/knn_bench.py
# --fast): dvcp/libdvcp_hip_A.so (A), the in-tree library (B) and, if present, dvcp/libdvcp_hip_C.so
# (C), alternating; then the selected parity tests on B.  Usage: tools/gpu_ab_micro.sh <tag> [pytest -k expr]
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
tag=${1:-abm}
kexpr=${2:-"knn or dfe"}
L=deepvcp-pointcloud-registration_amd/dvcp
if [ -f $L/libdvcp_hip_B.so ]; then cp $L/libdvcp_hip_B.so /tmp/libdvcp_hip_B.so; else cp $L/libdvcp_hip.so /tmp/libdvcp_hip_B.so; fi
vs="A B"
for v in C E F; do [ -f $L/libdvcp_hip_$v.so ] && vs="$vs $v"; done
for i in 1 2; do
  for v in $vs; do
    if [ $v = B ]; then cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so; else cp $L/libdvcp_hip_$v.so $L/libdvcp_hip.so; fi
    echo "== $v run $i" >> gpurun_out/${tag}.log
    DVCP_SKIP_ABI=1 timeout -k 10 200 python tools/knn_bench.py --fast >> gpurun_out/${tag}.log 2>&1 || exit $?
  done
done
cp /tmp/libdvcp_hip_B.so $L/libdvcp_hip.so
[ "$kexpr" = none ] && exit 0
timeout -k 10 400 python -u -m pytest tests -m gpu -k "$kexpr" -q --timeout 300 --timeout-method thread -rfs \
  > gpurun_out/${tag}_pytest.log 2>&1
