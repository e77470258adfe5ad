#!/bin/bash
# round 4: GPU suite + C3 bench after the select reduction and the trial grid change, then c3s bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_suite.sh r04p || exit $?
bash tools/r04_ab.sh r04p c3s 2 "-" || exit $?
