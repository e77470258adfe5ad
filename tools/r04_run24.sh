#!/bin/bash
# round 4: sanity after rebuilding the libraries from the committed sources: smoke, column-split tests, ASan GPU driver
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04zzz; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_abi_asan.py -k "column_split or step_graph or asan" -v --timeout 200 \
  --timeout-method thread > $OUT/t.log 2>&1; rc=$?; tail -3 $OUT/t.log; exit $rc
