#!/bin/bash
# Interleaved kbench trg A/B of two kbench builds (on the box): tools/ab_kbench_trg.sh <binA> <binB> [B...]
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
A=$1; Bb=$2; shift 2
for b in ${@:-8192 1024}; do
  for r in 1 2; do
    for v in $A $Bb; do echo "== B=$b $v r$r"; timeout -k 10 60 tools/$v $b trg | grep -E "direct|poly" || exit 1; done
  done
done
