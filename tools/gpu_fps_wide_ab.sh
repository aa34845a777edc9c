cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
DVCP_FPS_WIDE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "fps or e2e or sa_mlp_plain" > gpurun_out/fw_pytest.log 2>&1 || exit $?
DVCP_FPS_WIDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 > gpurun_out/fw_p1.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 > gpurun_out/fn_p1.log 2>&1 || exit $?
DVCP_FPS_WIDE=1 timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fw_p8.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fn_p8.log 2>&1
