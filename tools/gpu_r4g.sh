#!/bin/bash
# Round 4 G: matrix-core batch-statistics BN (sa2/sa3) parity first, then the kNN/DFE/CPG A/B of
# the stored builds (A = r3 .. F = bulk chunk test), the full GPU suite on the current tree (G),
# the bench, and the batch-statistics training step.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=deepvcp-pointcloud-registration_amd/dvcp
cp $L/libdvcp_hip.so /tmp/libdvcp_hip_G.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -rfs \
  -k "batch_stats or train_mode or fe_train or whole_model" > gpurun_out/r4g_train.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python tools/train_step_bench.py --train-fe --bn-train --steps 4 --warmup 2 > gpurun_out/r4g_train_bench.log 2>&1 || exit $?
bash tools/gpu_ab_micro.sh r4g_ab none || exit $?
cp /tmp/libdvcp_hip_G.so $L/libdvcp_hip.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfs > gpurun_out/r4g_pytest.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4g_bench.log 2> gpurun_out/r4g_bench.err
