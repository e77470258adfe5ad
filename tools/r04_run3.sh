#!/bin/bash
# round 4: GPU suite after the knob pruning, C3 bench, and the strong-scaling rank c3s (1024 rows)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/r04_suite.sh r04d || exit $?
bash tools/r04_ab.sh r04d c3s 1 "-" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r04d/prof_c3s" -o c3s -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c3s --no-cpu-baseline --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/r04d/prof_c3s.log" 2>&1
echo "rocprof rc $?"
