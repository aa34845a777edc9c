#!/bin/bash
# Stall breakdown of the kNN select and ball-query kernels: the micro-benchmarks, then one SQ
# PMC pass over each (wave cycles = active + waiting on counters + issue stalls).
ROOT="$GRAFT_REPO_ROOT"
TAG=${1:-r3s}
cd /tmp && export TMPDIR=/tmp && mkdir -p "$ROOT/gpurun_out"
timeout -k 10 120 python3 "$ROOT/tools/bq_bench.py" > "$ROOT/gpurun_out/${TAG}_bq_bench.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 -L > "$ROOT/gpurun_out/avail.txt" 2>&1
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$ROOT/gpurun_out/${TAG}_knn" -o run \
  -- python3 "$ROOT/tools/knn_bench.py" > "$ROOT/gpurun_out/${TAG}_knn.log" 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$ROOT/gpurun_out/${TAG}_bq" -o run \
  -- python3 "$ROOT/tools/bq_bench.py" > "$ROOT/gpurun_out/${TAG}_bq.log" 2>&1 || exit $?
C2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SMEM"
timeout -s KILL 150 rocprofv3 --pmc $C2 --output-format csv -d "$ROOT/gpurun_out/${TAG}_knn2" -o run \
  -- python3 "$ROOT/tools/knn_bench.py" > "$ROOT/gpurun_out/${TAG}_knn2.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc $C2 --output-format csv -d "$ROOT/gpurun_out/${TAG}_bq2" -o run \
  -- python3 "$ROOT/tools/bq_bench.py" > "$ROOT/gpurun_out/${TAG}_bq2.log" 2>&1
