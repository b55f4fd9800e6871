#!/bin/bash
# Round 5: the multi-rank round's code path at world 1 under torch.distributed.run (bench.py --world1-general: all-gather,
# plan and exchange as RCCL calls on the side streams), with its stages and host time, beside the one-launch round.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05dd}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --force-dist --world1-general --steps 100 --warmup 10 > $O/w1_general.json 2> $O/w1_general.err || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29542 bench.py --force-dist --steps 100 --warmup 10 > $O/w1_onelaunch.json 2> $O/w1_onelaunch.err
