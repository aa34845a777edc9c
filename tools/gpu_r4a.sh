cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfs --durations=15 > gpurun_out/r4a_pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc" >> gpurun_out/r4a_pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4a_bench.log 2> gpurun_out/r4a_bench.err
