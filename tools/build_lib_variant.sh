#!/bin/bash
# Build an A/B variant of libadmmlstm.so with one translation unit recompiled under extra flags:
#   tools/build_lib_variant.sh <name> <split3|kernels|host> <flags...>  ->  ablib/lib_<name>.so
# Load it with ADMM_LSTM_LIB=ablib/lib_<name>.so (tools/ab.sh).
set -e
cd "$(dirname "$0")/.."
name=$1; tu=$2; shift 2
C=admm-lstm_amd/admm_amd/csrc
make -s -C $C
mkdir -p ablib /tmp/abv_$name
objs=""
for t in kernels split3 host; do
  if [ "$t" = "$tu" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -Wall -Wno-unused-result "$@" \
      -c $C/admm_$t.hip -o /tmp/abv_$name/admm_$t.o
    objs="$objs /tmp/abv_$name/admm_$t.o"
  else
    objs="$objs $C/build/admm_$t.o"
  fi
done
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared $objs -o ablib/lib_$name.so -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
echo ablib/lib_$name.so
