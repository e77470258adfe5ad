#!/bin/bash
# N = 2 and 4 ranks of bench.py on the one GPU of a gpurun box (gloo, host-staged all-reduces): the N > 1
# path rehearsed, not a performance number.  usage (box): bash tools/rehearse_one_device.sh
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-rehearsal}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --one-device --dist-backend gloo --steps 6 --warmup 2 --no-cpu-baseline > $O/n2.json 2> $O/n2.err || { echo "n2 failed $?"; tail -20 $O/n2.err; exit 1; }
tail -c 400 $O/n2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --one-device --dist-backend gloo --steps 6 --warmup 2 --no-cpu-baseline > $O/n4.json 2> $O/n4.err || { echo "n4 failed $?"; tail -20 $O/n4.err; exit 1; }
tail -c 400 $O/n4.json
