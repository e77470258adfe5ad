#!/bin/bash
# A/B of env knobs on the C3 bench (GPU box): tools/r03_ab.sh OUTDIR "ENV1" "ENV2" ... ; each run
# under its own time limit, rounds interleaved; stops at the first failure
out=$1; shift
mkdir -p "$out"
for round in 1 2; do
  for cfg in "$@"; do
    tag=$(echo "$cfg" | tr ' =' '_-')
    env $cfg timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$out/ab_${tag}_r$round.json" 2> "$out/ab_${tag}_r$round.err" || exit 1
    python -c "import json,sys; d=json.load(open('$out/ab_${tag}_r$round.json')); print('$cfg', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['kernels'].items()})"
  done
done
