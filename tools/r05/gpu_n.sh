#!/bin/bash
# Round 5: the round's stage-timing events without the system-scope fence: bench's N=1 line (headline +
# round_world1, the driver's arguments), the world-1 round under torch.distributed.run, and its kernel trace (the
# gaps between scans at the timed rounds).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05n}
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err || exit 1
( export MASTER_ADDR=127.0.0.1 MASTER_PORT=29641 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w1_trace -o w1 -- \
    python3 $R/bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/w1_trace.json 2> $O/w1_trace.err )
