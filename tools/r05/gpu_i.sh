#!/bin/bash
# Round 5: BASELINE config 1, 4 MiB fp32, B=256, -r 1.0 (dense), 1 worker + 1 aggregator.
#  * bench.py at that shape (headline kernel, the world-1 round, cpu_baseline with 8 threads over 10 + 101 rounds and
#    the 1-thread figure);
#  * rocprofv3 --kernel-trace --stats of the same bench without the CPU legs (kernel durations against the events);
#  * ./omr_client -L 1 -r 1.0 -n 1048576 -c: the reference CLI's alg-bw lines (loopback, 1 worker + 1 aggregator).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05i}
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 > $O/c1.json 2> $O/c1.err || exit 1
timeout -k 10 120 omnireduce-rdma-demo_amd/bin/omr_client -L 1 -r 1.0 -n 1048576 -c > $O/client_L1.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o c1 --output-format csv -- \
  python3 $R/bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 --no-cpu > $O/c1_prof.json 2> $O/c1_prof.err
