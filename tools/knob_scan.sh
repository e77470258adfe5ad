#!/bin/bash
# bench.py --config $CFG under several knob settings (GPU box): final MSE, exponents, ms/step
# usage: CFG=c4g tools/knob_scan.sh OUTDIR "ENV1" "ENV2" ...
out=$1; shift; mkdir -p "$out"
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr ' =' '_-')
  env $cfg timeout -k 10 240 python -u bench.py --config ${CFG:-c3} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline \
      > "$out/scan_${tag}.json" 2> "$out/scan_${tag}.err" || { echo "$cfg failed"; exit 1; }
  python -c "import json; d=json.load(open('$out/scan_${tag}.json')); print('$cfg', d['ms_per_step'], d['final_train_mse'], d['line_search_k'])"
done
