#!/bin/bash
# A/B of one kernel-variant build, compiled ON the GPU box (keeps this container's CPU quiet for timing runs):
#   bash tools/ab_build_on_box.sh <tag> <name> <kernels|split3|host> <rounds> <pytest -k expr> <flags...>
# Builds the tree's library and ablib/lib_<name>.so (tools/build_lib_variant.sh), runs the GPU tests selected by
# the -k expression on both, then interleaved bench.py A/Bs at C3 (<rounds> rounds) and C5 (one round).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
TAG=$1; NAME=$2; TU=$3; R=$4; SEL=$5; shift 5
O=gpurun_out/$TAG; mkdir -p $O
set -o pipefail
timeout -k 10 600 make -s -C admm-lstm_amd/admm_amd/csrc -j4 > $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
timeout -k 10 600 bash tools/build_lib_variant.sh $NAME $TU "$@" >> $O/build.log 2>&1 || { tail -20 $O/build.log; exit 1; }
for lib in "" "ablib/lib_$NAME.so"; do
  ADMM_LSTM_LIB=$lib timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "$SEL" --timeout 200 \
    --timeout-method thread >> $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
done
grep -E "passed|failed" $O/tests.log
timeout -k 10 600 bash tools/ab.sh $R "base=" "$NAME=ADMM_LSTM_LIB=ablib/lib_$NAME.so" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
BENCH_ARGS="--config c5" timeout -k 10 400 bash tools/ab.sh 1 "base=" "$NAME=ADMM_LSTM_LIB=ablib/lib_$NAME.so" > $O/ab_c5.txt 2>&1 || { cat $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
