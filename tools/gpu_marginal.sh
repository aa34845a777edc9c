#!/bin/bash
# Marginal cost of each entry point under the bench's concurrency: run the bench with that entry
# issued twice per call (DVCP_DUP) and compare pairs/s with the plain run.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --steps 32 > gpurun_out/mc_$1.log 2>&1 || exit $?;
        echo "$1 $(grep -o '"value": [0-9.]*' gpurun_out/mc_$1.log)" >> gpurun_out/marginal.log; }
run base
for E in "$@"; do DVCP_DUP=$E run $E; done
run base2
