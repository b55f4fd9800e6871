#!/bin/bash
# Round-5 bench lines on one MI355X: config 2 (the headline, with round_world1), config 3, m=8
# (config 4's sum on one GPU), config 5 (host resident, N=1), the N>1 round at world 1 under torch.distributed.run;
# rocprofv3 kernel stats of configs 2 and 3, and PMC HBM traffic of configs 2 and 3.  Chained with &&.
set -e
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $GRAFT_REPO_ROOT/gpurun_out/smoke_r05.log 2>&1
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-bench_r05}
mkdir -p $O
cd $R
timeout -k 10 240 python3 bench.py > $O/c2.json 2> $O/c2.err
timeout -k 10 200 python3 bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round > $O/c3.json 2> $O/c3.err
timeout -k 10 200 python3 bench.py --workers 8 --no-cpu --no-round > $O/m8.json 2> $O/m8.err
timeout -k 10 200 python3 bench.py --host-resident --size-mib 4096 --density 0.49 --steps 5 --warmup 1 > $O/c5.json 2> $O/c5.err
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
timeout -k 10 300 python3 tools/pmc_traffic.py --out $O/pmc_r05.json --workdir $O/pmc_c2 > $O/pmc_c2.log 2>&1
timeout -k 10 300 python3 tools/pmc_traffic.py --out $O/pmc_c3_r05.json --workdir $O/pmc_c3 -- --size-mib 1024 \
  --block-size 1024 --density 0.0099 --steps 20 --warmup 5 --no-cpu --no-round > $O/pmc_c3.log 2>&1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-round > $O/c2_prof.json 2> $O/c2_prof.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o c3 --output-format csv -- \
  python3 $R/bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round > $O/c3_prof.json 2> $O/c3_prof.err
# the world-1 round's kernel trace beside its host laps (OMR_HOST_TRACE=2: CLOCK_MONOTONIC, rocprofv3's clock), and
# the round's kernels at config 4's shapes (their PMC traffic: tools/r04/gpu_r04_pmc_round.sh, a call of its own)
cd $R
( export MASTER_ADDR=127.0.0.1 MASTER_PORT=29641 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 OMR_HOST_TRACE=2 \
         OMR_HOST_TRACE_FILE=$O/w1_host_laps.txt
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/w1_trace -o w1 -- \
    python3 $R/bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/w1_trace.json 2> $O/w1_trace.err )
timeout -k 10 300 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
# round 5: the world-1 round in four stream layouts after a one-rank torch group (bench's N>1 set-up), and config 1
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  tools/round_inproc_r05.py --torch-group --reps 4 --json $O/inproc_group.json > $O/inproc_group.log 2>&1
timeout -k 10 300 python3 bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 > $O/c1.json 2> $O/c1.err
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 4 --json $O/inproc_nogroup.json > $O/inproc_nogroup.log 2>&1
