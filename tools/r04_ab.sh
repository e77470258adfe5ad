#!/bin/bash
# Round 4 A/B: bench lines of one config under several environment settings, interleaved rounds.
# usage: tools/r04_ab.sh TAG CONFIG ROUNDS "ENV1" "ENV2" ...   (ENV = space-separated VAR=VALUE, or "-" for none)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; CFG=$2; ROUNDS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=""; [ "$e" != "-" ] && envs="$e"
    env $envs timeout -k 10 240 python -u bench.py --config "$CFG" --no-cpu-baseline --steps 20 --warmup 5 \
      > "$OUT/ab_${CFG}_v${i}_r${r}.json" 2> "$OUT/ab_${CFG}_v${i}_r${r}.err"
    rc=$?
    [ $rc -eq 0 ] || { echo "stop: $e rc $rc"; tail -5 "$OUT/ab_${CFG}_v${i}_r${r}.err"; exit $rc; }
    python - "$OUT/ab_${CFG}_v${i}_r${r}.json" "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cls = {k: v['ms_per_step'] for k, v in d.get('kernels', {}).items()}
print(f"{sys.argv[2]:40s} {d['ms_per_step']:.4f} ms/step", cls)
PY
  done
done
