#!/bin/bash
# SQ counters of the isolated kernels (tools/kbench), one pass: bash tools/pmc_kbench.sh <tag> [kbench args]
set -e
TAG=$1; shift
R=$(pwd); OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o sq -- $R/tools/kbench "$@" > $OUT/sq.log 2>&1
cd $R; python3 tools/pmc_summary.py $OUT/sq > $OUT/sq_summary.txt
