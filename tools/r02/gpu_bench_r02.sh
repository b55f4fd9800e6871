#!/bin/bash
# Round-2 bench lines on one MI355X: config 2 (the headline), config 3, m=8 (config 4's sum on one GPU), config 5
# (host resident, N=1) and the N>1 round rehearsed at world 1 under torch.distributed.run; rocprofv3 kernel stats
# of config 2.  Each GPU step under its own time limit, chained with &&.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bench_r02
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py > $O/c2.json 2> $O/c2.err
timeout -k 10 200 python3 bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu > $O/c3.json 2> $O/c3.err
timeout -k 10 200 python3 bench.py --workers 8 --no-cpu > $O/m8.json 2> $O/m8.err
timeout -k 10 200 python3 bench.py --host-resident --size-mib 4096 --density 0.49 --steps 5 --warmup 1 > $O/c5.json 2> $O/c5.err
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
  python3 $R/bench.py --no-cpu > $O/c2_prof.json 2> $O/c2_prof.err
