#!/bin/bash
# round 4: row-block vs column-split sweep at the N = 2 and N = 4 strong-scaling ranks (4096, 2048 rows)
cd "$GRAFT_REPO_ROOT/tools" || exit 1
OUT=../gpurun_out/r04r; mkdir -p $OUT
for B in 4096 2048; do
  timeout -k 10 120 ./kbench_nc2 $B x 32 16 256 > $OUT/kb.$B.log 2>&1 || exit $?
  echo "B=$B"; grep -E "sweep rows|column" $OUT/kb.$B.log
done
