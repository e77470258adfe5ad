#!/bin/bash
# round 4: which of the step's extra sweep outputs costs the column split: ranges (atomics), tgt + G_x partials
cd "$GRAFT_REPO_ROOT/tools" || exit 1
OUT=../gpurun_out/r04v; mkdir -p $OUT
for B in 1024 4096; do
  for e in "KB_NONE=1" "KB_GX=1" "KB_GX=1 KB_NORANGE=1" "KB_GX=1 KB_NOTGT=1"; do
    env $e timeout -k 10 120 ./kbench $B x 32 16 256 > $OUT/kb.log 2>&1 || exit $?
    echo "B=$B $e"; grep -E "sweep rows|column split " $OUT/kb.log
  done
done
