#!/bin/bash
# round 4: column-split sweep check first (bounded), then the suite and c3s / c3 benches
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k column_split -v --timeout 120 --timeout-method thread > $OUT/cs.log 2>&1
rc=$?; tail -6 $OUT/cs.log; [ $rc -le 1 ] || exit $rc
bash tools/r04_ab.sh r04e c3s 2 "-" "ADMM_SWEEP_SPLIT_COLS=0" || exit $?
bash tools/r04_suite.sh r04e || exit $?
