cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_shard.py > gpurun_out/r4b_diag_shard.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k c5_head -v --timeout 280 --timeout-method thread -rfs > gpurun_out/r4b_c5.log 2>&1
