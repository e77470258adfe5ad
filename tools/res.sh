#!/bin/bash
# usage: tools_res.sh <file.hip>  -- per-kernel VGPR/occupancy/spill summary (gfx950)
cd /root/repo/admm-lstm_amd/admm_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/root/repo/include -c ${1:-admm_kernels.hip} -o /tmp/res.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|Spill|Occupancy" | paste - - - - - | sed -E 's/[a-z_]+.hip:[0-9]+:[0-9]+: remark: //g; s/\[-Rpass-analysis=kernel-resource-usage\]//g; s/_ZN4admm12_GLOBAL__N_1//; s/Function Name: //; s/Occupancy \[waves\/SIMD\]/occ/' | awk '{$1=$1; print}' | cut -c1-160
