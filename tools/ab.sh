#!/bin/bash
# Interleaved A/B of library builds on the GPU box (cdna_hip_programming.md rule 24: variants in
# alternating rounds).  usage: tools/ab.sh ROUNDS "label=ENV... " "label=ENV..." ...
#   e.g. tools/ab.sh 3 "new=" "old=ADMM_LSTM_LIB=ablib/lib_r02b.so"
# Each arm runs bench.py (C3 unless BENCH_ARGS says otherwise) and prints ms/step and the
# per-class kernel times.
R=${1:-3}; shift
for r in $(seq 1 $R); do
  for arm in "$@"; do
    label=${arm%%=*}; envs=${arm#*=}
    out=$(env $envs timeout -k 10 150 python3 bench.py --no-cpu-baseline $BENCH_ARGS 2>/dev/null | tail -1) || { echo "$label failed"; exit 1; }
    echo "$out" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
k = ' '.join(f'{c}={v[\"ms_per_step\"]:.3f}' for c, v in d['kernels'].items())
print(f'$label r$r {d[\"ms_per_step\"]:.3f} ms  {k}')"
  done
done
