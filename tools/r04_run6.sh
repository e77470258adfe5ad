#!/bin/bash
# round 4: column-split sweep phase timing (kbench_cst)
cd "$GRAFT_REPO_ROOT/tools" || exit 1
mkdir -p ../gpurun_out/r04g
timeout -k 10 120 ./kbench_cst 1024 x 32 16 256 > ../gpurun_out/r04g/cst.log 2>&1; rc=$?
grep -E -A2 "sweep column|column" ../gpurun_out/r04g/cst.log
exit $rc
