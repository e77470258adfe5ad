#!/bin/bash
# GPU suite, then an interleaved in-step A/B of the tree's library against ablib/lib_<base>.so at C3, c3s,
# c3q, c3h and C5 (tools/ab.sh).  usage (box): bash tools/ab_lib.sh <tag> <base> [rounds]
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
TAG=$1; BASE=$2; R=${3:-2}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 bash tools/gpu.sh $TAG tests || exit 1
(timeout -k 10 400 bash tools/ab.sh $R "new=" "$BASE=ADMM_LSTM_LIB=ablib/lib_$BASE.so" > $O/ab_c3.txt 2>&1) || exit 1
(BENCH_ARGS="--config c3s" timeout -k 10 300 bash tools/ab.sh $R "new=" "$BASE=ADMM_LSTM_LIB=ablib/lib_$BASE.so" > $O/ab_c3s.txt 2>&1) || exit 1
(BENCH_ARGS="--config c3q" timeout -k 10 300 bash tools/ab.sh $R "new=" "$BASE=ADMM_LSTM_LIB=ablib/lib_$BASE.so" > $O/ab_c3q.txt 2>&1) || exit 1
(BENCH_ARGS="--config c3h" timeout -k 10 300 bash tools/ab.sh $R "new=" "$BASE=ADMM_LSTM_LIB=ablib/lib_$BASE.so" > $O/ab_c3h.txt 2>&1) || exit 1
(BENCH_ARGS="--config c5" timeout -k 10 400 bash tools/ab.sh 1 "new=" "$BASE=ADMM_LSTM_LIB=ablib/lib_$BASE.so" > $O/ab_c5.txt 2>&1) || exit 1
cat $O/ab_c3.txt $O/ab_c3s.txt $O/ab_c3q.txt $O/ab_c3h.txt $O/ab_c5.txt
