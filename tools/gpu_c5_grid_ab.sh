cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
L=$PWD/deepvcp-pointcloud-registration_amd/dvcp
for i in 1 2; do for v in g768 g512; do
  echo "== $v run $i" >> gpurun_out/r6al_c5_grid.log
  DVCP_LIB_PATH=$L/libdvcp_hip_$v.so timeout -k 10 200 python bench.py --config c5 --steps 30 --warmup 5 --no-cpu-baseline >> gpurun_out/r6al_c5_grid.log 2>&1 || exit 1
done; done
