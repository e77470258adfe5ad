#!/bin/bash
# kbench variant with admm_kernels.hip compiled under extra flags: tools/build_variant_k.sh <name> <flags...>
set -e
cd "$(dirname "$0")"
name=$1; shift
C=../admm-lstm_amd/admm_amd/csrc
make -s -C $C
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include "$@" -c $C/admm_kernels.hip -o /tmp/k_$name.o
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include "$@" -c kbench.hip -o /tmp/kbench.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/kbench.o /tmp/k_$name.o $C/build/admm_split3.o -o kbench_$name
