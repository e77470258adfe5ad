#!/bin/bash
# Round 4: the GPU suite (records under gpurun_out/<tag>/parity), then a C3 bench line (no CPU
# baseline).  Stops at the first step that faults, aborts or times out.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r04b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ADMM_PARITY_OUT=$OUT/parity timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -4 "$OUT/gpu_tests.log"
[ $rc -le 1 ] || { echo "stop: tests rc $rc"; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?
tail -c 1500 "$OUT/bench_c3.json"
exit $rc
