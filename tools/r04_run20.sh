#!/bin/bash
# round 4: the host-ASan driver alone (it went silent for 180 s in r04w), then the rest of the GPU suite and bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04x; mkdir -p $OUT
(cd admm-lstm_amd/admm_amd && ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:halt_on_error=1 LSAN_OPTIONS=suppressions=$GRAFT_REPO_ROOT/tests/native/lsan.supp:print_suppressions=0 timeout -k 10 150 ./abi_asan gpu > ../../$OUT/asan_gpu.log 2>&1); rc=$?
echo "asan driver rc $rc"; tail -5 $OUT/asan_gpu.log
[ $rc -eq 0 ] || exit $rc
ADMM_PARITY_OUT=$OUT/parity timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > $OUT/gpu_tests.log 2>&1
rc=$?; tail -4 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
python -c "import json;d=json.loads(open('$OUT/bench_c3.json').read().strip().splitlines()[-1]);print('C3',d['value'],d['ms_per_step'],{k:v['ms_per_step'] for k,v in d['kernels'].items()})"
bash tools/r04_ab.sh r04x c3s 1 "-" || exit $?
bash tools/r04_ab.sh r04x c3h 1 "-" || exit $?
