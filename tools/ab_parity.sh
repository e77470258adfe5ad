#!/bin/bash
# A/B of library builds on the bench trajectory's arithmetic drift (GPU box): for each arm, the forced-decision
# 25-step C3 run against the reference and the fp64 oracle (tests/test_gpu_trajectory.py, record under
# gpurun_out/<tag>/<label>/parity_c3_25_forced.json), then interleaved bench.py timings (tools/ab.sh).
# usage: bash tools/ab_parity.sh <tag> <rounds> "label=ENV..." ...   (ENV e.g. ADMM_LSTM_LIB=ablib/lib_x.so)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for arm in "$@"; do
  label=${arm%%=*}; envs=${arm#*=}
  mkdir -p $O/$label
  env $envs ADMM_PARITY_OUT=$O/$label timeout -k 10 400 python -u -m pytest tests/test_gpu_trajectory.py -q \
    -k forced --timeout 300 --timeout-method thread > $O/$label/traj.log 2>&1
  rc=$?
  echo "$label: forced trajectory rc $rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 900 bash tools/ab.sh $R "$@" > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
