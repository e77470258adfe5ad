#!/bin/bash
# round 4: two-group column split at 4096 rows: bitwise tests, then per-rank bench lines at N = 2, 4, 8 (c3h, c3q, c3s)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04s; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "column_split or step_graph" -v --timeout 200 \
  --timeout-method thread > $OUT/cs.log 2>&1
rc=$?; tail -4 $OUT/cs.log; [ $rc -le 1 ] || exit $rc
bash tools/r04_ab.sh r04s c3h 1 "-" "ADMM_SWEEP_SPLIT_COLS=0" || exit $?
bash tools/r04_ab.sh r04s c3q 1 "-" "ADMM_SWEEP_SPLIT_COLS=0" || exit $?
bash tools/r04_ab.sh r04s c3s 1 "-" || exit $?
