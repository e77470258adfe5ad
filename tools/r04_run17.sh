#!/bin/bash
# round 4: column-split phase timing with and without the step's extra outputs (KB_GX=1), 1024 rows
cd "$GRAFT_REPO_ROOT/tools" || exit 1
OUT=../gpurun_out/r04u; mkdir -p $OUT
for gx in 0 1; do
  if [ $gx = 1 ]; then e="KB_GX=1"; else e="KB_NONE=1"; fi
  env $e timeout -k 10 120 ./kbench_cst 1024 x 32 16 256 > $OUT/cst.gx$gx.log 2>&1 || exit $?
  echo "gx=$gx"; grep -E "column" $OUT/cst.gx$gx.log
done
