cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/diag_shard.py > gpurun_out/r4e_diag_shard.log 2>&1 || exit $?
bash tools/gpu_micro_pmc.sh r4e_pmc || exit $?
bash tools/gpu_ab_micro.sh r4e_ab "knn"
