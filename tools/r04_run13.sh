#!/bin/bash
# round 4 final traces: rocprofv3 kernel trace of the default bench command (C3) and of c3s, each beside its bench line
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04q; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for cfg in c3 c3s; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$cfg" -o $cfg -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --config $cfg --no-cpu-baseline > "$GRAFT_REPO_ROOT/$OUT/bench_under_rocprof_$cfg.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_$cfg.err"
  rc=$?; echo "rocprof $cfg rc $rc"; [ $rc -eq 0 ] || exit $rc
done
