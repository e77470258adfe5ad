#!/bin/bash
# round 4: c3s bench lines, its rocprofv3 kernel trace, smoke, and the default bench (C3 with the CPU baseline)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04j}; OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/r04_ab.sh $TAG c3s 2 "-" || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c3s" -o c3s -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --config c3s --no-cpu-baseline --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/$OUT/prof_c3s.log" 2>&1)
rc=$?; echo "rocprof rc $rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err; rc=$?
tail -c 2500 $OUT/bench_default.json; exit $rc
