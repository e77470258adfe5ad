#!/bin/bash
# round 4 final tree: rocprofv3 kernel trace of the c3s bench command beside its bench line
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04f2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c3s" -o c3s -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c3s --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof_c3s.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_c3s.err"
rc=$?; echo "rocprof c3s rc $rc"; exit $rc
