#!/bin/bash
# round 4: N = 2 bench path rehearsed on one GPU with the final tree (two ranks' column-split sweeps contend for the
# CUs here, so the entry consensus / row-block fallback path runs; not a performance number)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/r04zz; mkdir -p $OUT
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 \
  bench.py --gpus 2 --one-device --steps 5 --warmup 2 --no-cpu-baseline > $OUT/n2.json 2> $OUT/n2.err
rc=$?; echo "rc $rc"; tail -c 600 $OUT/n2.json; grep -i -E "error|nonfinite|warn" $OUT/n2.err | head -5; exit $rc
