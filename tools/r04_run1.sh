#!/bin/bash
# round 4, first f16 check: the GPU suite, then C3 and C5 A/B of the h-side gradient modes
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_suite.sh r04c || exit $?
bash tools/r04_ab.sh r04c c3 2 "-" "ADMM_ATR_F16=0" "ADMM_ATR_F16=0 ADMM_ATR_PIECES=2" || exit $?
bash tools/r04_ab.sh r04c c5 1 "-" "ADMM_ATR_F16=0" "ADMM_ATR_F16=0 ADMM_ATR_PIECES=2" || exit $?
