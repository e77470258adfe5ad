#!/bin/bash
# round 4: sweep extra-output isolation (kbench), then the GPU suite + C3 bench and c3s / c3h lines on the same box
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_run18.sh || exit $?
bash tools/r04_suite.sh r04w || exit $?
bash tools/r04_ab.sh r04w c3s 1 "-" || exit $?
bash tools/r04_ab.sh r04w c3h 1 "-" || exit $?
