#!/bin/bash
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "dfe or e2e_c3" > gpurun_out/pytest_sel.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --stage-report > gpurun_out/bench1.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_xcd_FETCH_SIZE" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --inflight 1 --steps 4 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_xcd.log" 2>&1
