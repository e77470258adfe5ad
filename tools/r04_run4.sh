#!/bin/bash
# round 4: column-split sweep and step-graph checks first (bounded), then c3s / c3 A/B, the c5g
# fixture (oracle on the device) and the suite
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "column_split or step_graph" -v --timeout 150 \
  --timeout-method thread > $OUT/cs.log 2>&1
rc=$?; tail -12 $OUT/cs.log; [ $rc -le 1 ] || exit $rc
bash tools/r04_ab.sh r04e c3s 2 "-" "ADMM_SWEEP_SPLIT_COLS=0" "ADMM_GRAPH=1" || exit $?
bash tools/r04_ab.sh r04e c3 1 "-" "ADMM_GRAPH=1" || exit $?
timeout -k 10 600 python -u tools/make_c5g.py $OUT/c5g.npz > $OUT/c5g.log 2>&1
rc=$?; tail -5 $OUT/c5g.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_suite.sh r04e || exit $?
