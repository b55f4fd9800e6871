#!/bin/bash
# Round-3 bench lines on one MI355X: config 2 (the headline, with round_world1), config 3, m=8
# (config 4's sum on one GPU), config 5 (host resident, N=1), the N>1 round at world 1 under torch.distributed.run;
# rocprofv3 kernel stats of config 2 and its PMC HBM traffic.  Each GPU step under its own time limit, chained with &&.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-bench_r03}
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py > $O/c2.json 2> $O/c2.err
timeout -k 10 200 python3 bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round > $O/c3.json 2> $O/c3.err
timeout -k 10 200 python3 bench.py --workers 8 --no-cpu --no-round > $O/m8.json 2> $O/m8.err
timeout -k 10 200 python3 bench.py --host-resident --size-mib 4096 --density 0.49 --steps 5 --warmup 1 > $O/c5.json 2> $O/c5.err
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
timeout -k 10 300 python3 tools/pmc_traffic.py --out $O/pmc_r03.json --workdir $O/pmc_c2 > $O/pmc_c2.log 2>&1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 python3 \
  tools/pmc_traffic.py --out $O/pmc_dist_w1_r03.json --workdir $O/pmc_w1 -- --force-dist --steps 20 --warmup 5 \
  > $O/pmc_w1.log 2>&1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-round > $O/c2_prof.json 2> $O/c2_prof.err
