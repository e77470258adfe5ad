#!/bin/bash
# x-trial grid scan with the g gate in the per-candidate regime (tools/kbench trg, KB_NB0), on the box.
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
for b in 1024 2048; do
  for nb in 64 128 192 256 384 512; do
    echo "== B=$b nb0=$nb"
    KB_NB0=$nb KB_NB1=$nb timeout -k 10 60 tools/kbench $b trg | grep -E "g direct|all poly" || exit 1
  done
done
