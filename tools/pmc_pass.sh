#!/bin/bash
# One rocprofv3 counter pass over a short bench.py run (one counter group per run; see
# MI355X_MICROARCH.md for the per-block limits):
#   bash tools/pmc_pass.sh <tag> <COUNTER> [COUNTER...]     (env passes through, e.g. ADMM_LSTM_LIB)
# -> gpurun_out/<tag>/summary.txt (per-kernel sums, tools/pmc_summary.py)
set -e
TAG=$1; shift
R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/run.log 2>&1
cd $R; python3 tools/pmc_summary.py $OUT/pmc > $OUT/summary.txt
