#!/bin/bash
# SQ counters of every kernel of a short bench.py run (one rocprofv3 pass):
#   bash tools/pmc_sq_bench.sh <tag>       (env passes through, e.g. ADMM_TRIAL_MX=0)
set -e
TAG=$1
R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o sq -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1
cd $R; python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt
