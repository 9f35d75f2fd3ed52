#!/bin/bash
# VGPR / LDS / scratch / occupancy of the pipeline kernels for a set of -D flags (measurement aid).
#   tools/kres.sh "-DFLAG ..."
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$R/include -I$R/gol-distributed-final_amd/csrc -mllvm -amdgpu-atomic-optimizer-strategy=None $1 \
  --cuda-device-only -c -Rpass-analysis=kernel-resource-usage $R/gol-distributed-final_amd/csrc/gol_kernels.hip \
  -o /tmp/kres.o 2>&1 | grep -A12 "Function Name: .*pipe_kernel" | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" | sed 's/.*remark: //'
