#!/bin/bash
# round 4: register-resident B in the column-split producer: bitwise tests, phase timing, c3s bench
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "column_split or step_graph" -v --timeout 150 \
  --timeout-method thread > $OUT/cs.log 2>&1
rc=$?; tail -10 $OUT/cs.log; [ $rc -le 1 ] || exit $rc
(cd tools && timeout -k 10 120 ./kbench_cst 1024 x 32 16 256 > ../$OUT/cst.log 2>&1); rc=$?
grep -E "sweep|column" $OUT/cst.log; [ $rc -eq 0 ] || exit $rc
bash tools/r04_ab.sh r04l c3s 2 "-" || exit $?
