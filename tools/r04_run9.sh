#!/bin/bash
# round 4: cooperative launch of the column-split sweep (A/B), and the N = 2 bench path rehearsed on one GPU
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04k; mkdir -p $OUT
for v in 0 1; do
  (cd tools && ADMM_SWEEP_COOP=$v timeout -k 10 120 ./kbench 1024 x 32 16 256 > ../$OUT/kb_coop$v.log 2>&1) || exit $?
  echo "coop=$v"; grep -E "column" $OUT/kb_coop$v.log
done
bash tools/r04_ab.sh r04k c3s 2 "-" "ADMM_SWEEP_COOP=1" || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --one-device --steps 5 --warmup 2 --no-cpu-baseline > $OUT/n2_rehearsal.json 2> $OUT/n2_rehearsal.err
rc=$?; tail -c 1500 $OUT/n2_rehearsal.json; tail -3 $OUT/n2_rehearsal.err; exit $rc
