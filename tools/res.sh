#!/bin/bash
# usage: tools/res.sh [file.hip] [extra hipcc flags...] -- per-kernel VGPR/occupancy/spill summary (gfx950)
cd /root/repo/admm-lstm_amd/admm_amd/csrc
F=${1:-admm_kernels.hip}; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I/root/repo/include "$@" -c $F -o /tmp/res.o -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs:|Spill|Occupancy" | sed -E 's/.*remark: +//; s/ \[-Rpass-analysis=kernel-resource-usage\]//; s/_ZN4admm12_GLOBAL__N_1//' | paste - - - - - - | awk '{$1=$1; print}' | cut -c1-170
