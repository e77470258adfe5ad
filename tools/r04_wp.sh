#!/bin/bash
# Round 4: the weight-phase tests (perturbed goldens, same-operand gradient GEMM accuracy) at the
# default h-side gradient pieces and at ATR_PIECES=3; pytest failures (rc 1) do not stop the script,
# anything else (fault, abort, timeout) does.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-r04a}
mkdir -p "$OUT"
run() {   # tag, env...
  local tag=$1; shift
  env "$@" ADMM_PARITY_OUT=$OUT/parity_$tag timeout -k 10 400 python -u -m pytest tests/test_gpu_weight_phase.py -v \
    --timeout 300 --timeout-method thread > "$OUT/wp_$tag.log" 2>&1
  local rc=$?
  tail -3 "$OUT/wp_$tag.log"
  [ $rc -le 1 ] || { echo "stop: rc $rc"; exit $rc; }
}
run f16 ADMM_ATR_F16=1
run s3 ADMM_ATR_F16=0
