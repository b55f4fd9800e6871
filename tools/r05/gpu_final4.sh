#!/bin/bash
# Round 5's last bench lines after the N>1 timed region's barrier-first close (the library is final3's): the driver's
# N=1 arguments, the default run (cpu_baseline, round_world1), and the world-1 round as its own line.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final4
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err || exit 1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --force-dist --steps 20 --warmup 5 > $O/dist_w1_k20.json 2> $O/dist_w1_k20.err || exit 1
