#!/bin/bash
# Build an A/B variant library: one source recompiled with extra -D flags, linked with the in-tree
# objects of every other source, into dvcp/libdvcp_hip_<name>.so (loaded by tools/gpu_ab_*.sh
# through DVCP_LIB_PATH; the in-tree library is not touched).  Delete the variants before a round
# ends (they travel with every gpurun call).
#   tools/build_variant.sh <name> <source stem, e.g. dfe_mfma> [-DNAME=VALUE ...]
set -e
name=$1; stem=$2; shift 2
cd "$(dirname "$0")/../deepvcp-pointcloud-registration_amd"
make -s -j8
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function -I../include"
case $stem in
  fps) EXTRA="-mllvm -amdgpu-promote-alloca-to-vector-limit=2048 -fno-slp-vectorize" ;;
  knn_tiled) EXTRA="-mllvm -amdgpu-promote-alloca-to-vector-limit=2048" ;;
  sa_bn) EXTRA="-mllvm -amdgpu-promote-alloca-to-vector-limit=4096" ;;
  *) EXTRA="" ;;
esac
mkdir -p build/var
/opt/rocm/bin/hipcc $HIPFLAGS $EXTRA "$@" -c csrc/$stem.hip -o build/var/${stem}_$name.o
objs=$(ls build/*.o | grep -v "build/$stem.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -mcode-object-version=5 -o dvcp/libdvcp_hip_$name.so \
  $objs build/var/${stem}_$name.o
echo "built dvcp/libdvcp_hip_$name.so ($stem $*)"
