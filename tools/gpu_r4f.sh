cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=deepvcp-pointcloud-registration_amd/dvcp
timeout -k 10 120 python tools/cpg_diag.py --lib $L/libdvcp_hip_D.so > gpurun_out/r4f_cpg_diag.log 2>&1 || exit $?
bash tools/gpu_ab_micro.sh r4f_ab none || exit $?
cp $L/libdvcp_hip_E.so $L/libdvcp_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs > gpurun_out/r4f_E_pytest.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4f_E_bench.log 2> gpurun_out/r4f_E_bench.err
rc=$?
[ $rc -eq 0 ] || exit $rc
if [ -f $L/libdvcp_hip_F.so ]; then
  cp $L/libdvcp_hip_F.so $L/libdvcp_hip.so
  timeout -k 10 400 python -u -m pytest tests -m gpu -k "knn or c3_pair_vs_oracle" -q --timeout 300 \
    --timeout-method thread -rfs > gpurun_out/r4f_F_pytest.log 2>&1
fi
