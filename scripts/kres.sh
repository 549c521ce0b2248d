#!/bin/bash
# Register / LDS / spill report of the step kernels of one model specialisation (default 1 = G1).
cd "$(dirname "$0")/../mjlab-1_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fno-hip-fp32-correctly-rounded-divide-sqrt \
  -DMJX_SPEC_ID=${1:-1} -c -o /tmp/kres.o spec.hip -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|AGPRs|Spill|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //'
