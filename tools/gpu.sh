#!/bin/bash
# One parameterised GPU-box runner (replaces round 4's one-off tools/r04_run*.sh scripts).
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# Steps, run in order; the script stops at the first step that fails, aborts or times out:
#   tests[:<pytest -k expr>]   GPU suite (records under gpurun_out/<tag>/parity)
#   smoke                      __graft_entry__.smoke()
#   bench:<cfg>[:<args>]       bench.py --config <cfg> --no-cpu-baseline <args>  -> bench_<cfg>.json
#   benchcpu:<cfg>             bench.py --config <cfg> (with the CPU baseline)   -> bench_<cfg>_cpu.json
#   trace:<cfg>                rocprofv3 --kernel-trace --stats of the bench command beside its bench line
#   traffic:<cfg>              FETCH_SIZE and WRITE_SIZE passes (one each)       -> pmc_<cfg>.json
#   mfma:<cfg>                 one SQ/GRBM pass for MFMA-busy                    -> sq_<cfg>.json
#   list                       rocprofv3 -L (the counters this box offers)       -> counters.txt
# Extra bench arguments for every bench-driven step: BENCH_ARGS (env).  Env passes through
# (e.g. ADMM_LSTM_LIB for an A/B build).
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.." || exit 1
R=$(pwd)
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

fail() { echo "stop: $1 (rc $2)"; exit "$2"; }

counters_list() {
  [ -s "$OUT/counters.txt" ] || (cd /tmp && timeout -s KILL 90 rocprofv3 -L > "$OUT/counters.txt" 2>&1)
}

for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  cfg=${rest%%:*}; extra=${rest#*:}; [ "$extra" = "$rest" ] && extra=""
  echo "== $step  $(date +%T)"
  case $kind in
    tests)
      sel=(); [ -n "$rest" ] && sel=(-k "$rest")
      ADMM_PARITY_OUT=$OUT/parity timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 \
        --timeout-method thread "${sel[@]}" > "$OUT/gpu_tests.log" 2>&1
      rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || fail tests $rc ;;
    smoke)
      timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1
      rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || fail smoke $rc ;;
    bench)
      timeout -k 10 300 python -u bench.py --config "$cfg" --no-cpu-baseline $extra $BENCH_ARGS \
        > "$OUT/bench_$cfg.json" 2> "$OUT/bench_$cfg.err"
      rc=$?; tail -c 600 "$OUT/bench_$cfg.json"; echo; [ $rc -eq 0 ] || fail bench $rc ;;
    benchcpu)
      timeout -k 10 900 python -u bench.py --config "$cfg" $BENCH_ARGS \
        > "$OUT/bench_${cfg}_cpu.json" 2> "$OUT/bench_${cfg}_cpu.err"
      rc=$?; tail -c 600 "$OUT/bench_${cfg}_cpu.json"; echo; [ $rc -eq 0 ] || fail benchcpu $rc ;;
    trace)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$cfg" -o ks -- \
        python3 "$R/bench.py" --config "$cfg" --no-cpu-baseline $BENCH_ARGS \
        > "$OUT/bench_under_rocprof_$cfg.json" 2> "$OUT/trace_$cfg.err")
      rc=$?; [ $rc -eq 0 ] || fail trace $rc
      find "$OUT/trace_$cfg" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$cfg.csv" \; ;;
    traffic)
      for c in FETCH_SIZE WRITE_SIZE; do
        (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${cfg}_$c" -o p -- \
          python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
          > "$OUT/pmc_${cfg}_$c.log" 2>&1)
        rc=$?; [ $rc -eq 0 ] || fail "traffic $c" $rc
      done
      python3 tools/pmc_to_json.py "$OUT/pmc_${cfg}_FETCH_SIZE" "$OUT/pmc_${cfg}_WRITE_SIZE" "$OUT/pmc_$cfg.json" \
        "$cfg, bench.py --config $cfg --steps 2 --warmup 1, rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes" \
        || fail pmc_to_json 1 ;;
    mfma)
      counters_list
      want=(SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_F32
            SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE GRBM_COUNT)
      have=(); nsq=0; ngr=0
      for c in "${want[@]}"; do
        grep -qw "$c" "$OUT/counters.txt" || continue
        case $c in SQ_*) [ $nsq -lt 8 ] || continue; nsq=$((nsq+1));; GRBM_*) [ $ngr -lt 2 ] || continue; ngr=$((ngr+1));; esac
        have+=("$c")
      done
      echo "counters: ${have[*]}"
      (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc "${have[@]}" --output-format csv -d "$OUT/sq_$cfg" -o p -- \
        python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS \
        > "$OUT/sq_$cfg.log" 2>&1)
      rc=$?; [ $rc -eq 0 ] || fail mfma $rc
      python3 tools/pmc_summary.py "$OUT/sq_$cfg" > "$OUT/sq_${cfg}_summary.txt"
      python3 tools/pmc_to_json.py --sq "$OUT/sq_$cfg" "$OUT/sq_$cfg.json" \
        "$cfg, bench.py --config $cfg --steps 2 --warmup 1, rocprofv3 --pmc ${have[*]}" || fail sq_to_json 1 ;;
    list)
      counters_list; grep -iE 'MFMA|BUSY|GRBM_GUI|GRBM_COUNT' "$OUT/counters.txt" | head -40 ;;
    *) fail "unknown step $step" 2 ;;
  esac
done
echo "== done $(date +%T)"
