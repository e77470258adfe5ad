#!/bin/bash
# round 4: GPU suite after the knob pruning, then C3 bench
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_suite.sh r04d || exit $?
