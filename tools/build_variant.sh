#!/bin/bash
# Build kbench variants with admm_split3.hip compiled under extra flags:
#   tools/build_variant.sh <name> <flags...>   ->  tools/kbench_<name>
set -e
cd "$(dirname "$0")"
name=$1; shift
C=../admm-lstm_amd/admm_amd/csrc
make -s -C $C
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include "$@" -c $C/admm_split3.hip -o /tmp/s3_$name.o
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -c kbench.hip -o /tmp/kbench.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/kbench.o $C/build/admm_kernels.o /tmp/s3_$name.o -o kbench_$name
