#!/bin/bash
# round 4: how long the host-ASan driver takes on the box, alone and twice
cd "$GRAFT_REPO_ROOT/admm-lstm_amd/admm_amd" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04y; mkdir -p $OUT
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1 LSAN_OPTIONS=suppressions=$GRAFT_REPO_ROOT/tests/native/lsan.supp:print_suppressions=0
for i in 1 2; do
  s=$(date +%s.%N)
  timeout -k 10 170 ./abi_asan gpu > $OUT/asan_$i.log 2>&1; rc=$?
  e=$(date +%s.%N); echo "run $i rc $rc $(echo "$e - $s" | bc) s"; grep -E "context|ok|FAIL" $OUT/asan_$i.log
  [ $rc -eq 0 ] || exit $rc
done
