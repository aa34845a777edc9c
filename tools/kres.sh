#!/bin/bash
# Kernel resource usage (VGPRs, AGPRs, scratch, LDS, occupancy) of one csrc/*.hip file for gfx950.
# Usage: tools/kres.sh csrc/dfe_mfma.hip [extra hipcc flags] | grep -A8 <kernel substring>
cd "$(dirname "$0")/../deepvcp-pointcloud-registration_amd" || exit 1
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -mcode-object-version=5 -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -I../include --offload-device-only -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|LDS Size|Occupancy" \
  | sed -e 's/.*remark: //'
