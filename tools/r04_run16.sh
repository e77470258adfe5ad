#!/bin/bash
# round 4: row-block vs column-split sweep with the step's extra outputs (tgt, G_x partials, ranges: KB_GX=1) and without
cd "$GRAFT_REPO_ROOT/tools" || exit 1
OUT=../gpurun_out/r04t; mkdir -p $OUT
for B in 4096 2048 1024; do
  for gx in 0 1; do
    if [ $gx = 1 ]; then e="KB_GX=1"; else e="KB_NONE=1"; fi
    env $e timeout -k 10 120 ./kbench $B x 32 16 256 > $OUT/kb.$B.gx$gx.log 2>&1 || exit $?
    echo "B=$B gx=$gx"; grep -E "sweep rows|column split " $OUT/kb.$B.gx$gx.log
  done
done
