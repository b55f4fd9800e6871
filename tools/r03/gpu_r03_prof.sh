#!/bin/bash
# Round 3 profiles: rocprofv3 kernel stats of the headline bench (config 2), the headline's PMC traffic, the PMC
# traffic of the world-1 round's worker scan (which writes the shard sums itself), and the round's kernels at
# config-4 shapes (tools/pmc_round.py).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03c}
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
  python3 $R/bench.py --no-cpu > $O/c2_prof.json 2> $O/c2_prof.err && \
cd $R && \
timeout -k 10 300 python3 tools/pmc_traffic.py --out $O/pmc_c2_r03.json --workdir $O/pmc_c2 > $O/pmc_c2.log 2>&1 && \
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 python3 \
  tools/pmc_traffic.py --out $O/pmc_dist_w1_r03.json --workdir $O/pmc_w1 -- --force-dist --steps 20 --warmup 5 \
  > $O/pmc_w1.log 2>&1 && \
timeout -k 10 900 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
