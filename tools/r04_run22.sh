#!/bin/bash
# round 4 final: the GPU suite, smoke, C3 bench (default command, with the CPU baseline), c3s / c3h / c3q lines
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04z; mkdir -p $OUT
ADMM_PARITY_OUT=$OUT/parity timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
python -c "import json;d=json.loads(open('$OUT/bench_default.json').read().strip().splitlines()[-1]);print('C3',d['value'],d['ms_per_step'],{k:v['ms_per_step'] for k,v in d['kernels'].items()})"
for c in c3s c3h c3q; do bash tools/r04_ab.sh r04z $c 1 "-" || exit $?; done
