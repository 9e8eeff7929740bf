#!/bin/bash
# VGPR / AGPR / spill / LDS / occupancy report of the kernels in one csrc file (gfx950)
# usage: tools/resource_usage.sh gemm_bf16.hip [kernel-name-filter]
cd "$(dirname "$0")/../sequential-variational-autoencoder_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I. -x hip -c "$1" -o /tmp/ru.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy|LDS Size" |
  sed 's/.*remark: //' | paste - - - - - - - - | grep -E "${2:-.}" | sed 's/\t/ | /g'
