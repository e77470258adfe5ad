#!/bin/bash
# round 4: k_select timing (tools/kbench "sel"): round-3 kernel (kbench_old) against the per-slot transposed wave
# reduction (kbench_new); the trial kernels' grid at c3s and C3 (KB_NB); then the dist tests (fused vs all-reduced selection)
cd "$GRAFT_REPO_ROOT/tools" || exit 1
OUT=../gpurun_out/r04n; mkdir -p $OUT
for b in kbench_old kbench_new; do
  for B in 1024 8192; do
    timeout -k 10 60 ./$b $B sel 32 16 256 > $OUT/$b.$B.log 2>&1 || exit $?
    echo "$b B=$B"; grep select $OUT/$b.$B.log | awk 'NR%3==0'
  done
done
for B in 1024 8192; do for nb in 512 256 128; do
  KB_NB=$nb timeout -k 10 120 ./kbench $B tr 32 16 256 > $OUT/tr.$B.$nb.log 2>&1 || exit $?
  echo "trials B=$B nb=$nb"; grep trial $OUT/tr.$B.$nb.log | tail -2
done; done
cd .. && timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread > $OUT/dist.log 2>&1; rc=$?
tail -8 $OUT/dist.log; exit $rc
