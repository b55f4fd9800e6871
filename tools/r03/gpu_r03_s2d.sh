#!/bin/bash
# Round 3, second session: bench's round_world1 now made behind a one-rank torch nccl group (as at N>1); kernel traces
# of the world-1 round with and without that group (which queue / stream each kernel ran on); the PMC HBM traffic of
# the round's kernels at config-4 shapes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2d}
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err && \
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err && \
cd /tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_group -o w1 --output-format csv -- \
  python3 $R/tools/round_w1.py --steps 40 > $O/trace_group.json 2> $O/trace_group.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_nogroup -o w1 --output-format csv -- \
  python3 $R/tools/round_w1.py --steps 40 --no-group > $O/trace_nogroup.json 2> $O/trace_nogroup.err && \
cd $R && \
timeout -k 10 600 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
