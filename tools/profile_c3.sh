#!/bin/bash
# Round profile of the C3 bench: kernel trace + stats, then FETCH_SIZE / WRITE_SIZE PMC passes
# (one counter group per run, MI355X_MICROARCH.md HBM section).  Run on the GPU box from the
# repo root:  bash tools/profile_c3.sh <tag>
set -e
TAG=${1:-r01c}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/ks_bench.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o w -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1
cd $R
python3 tools/pmc_to_json.py $OUT/fetch $OUT/write $OUT/pmc_c3.json "C3 (B=8192 T=32 D=16 H=256), bench.py --steps 2 --warmup 1, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes"
find $OUT/ks -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
echo done
