#!/bin/bash
# Build the isolated kernel benchmark against the library's kernel translation unit.
set -e
cd "$(dirname "$0")"
make -s -C ../admm-lstm_amd/admm_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -c kbench.hip -o /tmp/kbench.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/kbench.o ../admm-lstm_amd/admm_amd/csrc/build/admm_kernels.o ../admm-lstm_amd/admm_amd/csrc/build/admm_split3.o -o kbench
