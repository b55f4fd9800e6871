#!/bin/bash
# Round 3, second session: why the world-1 round made in-process (bench's round_world1, tools/round_w1.py) takes
# ~140 us per round when the same round under torch.distributed.run takes ~60: stream -> hardware-queue mapping
# variants, alternated twice; then the PMC HBM traffic of the round's kernels at config-4 shapes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2c}
mkdir -p $O
cd $R
for rep in 1 2; do
  timeout -k 10 120 python3 tools/round_w1.py > $O/plain_$rep.json 2> $O/plain_$rep.err || exit 1
  timeout -k 10 120 python3 tools/round_w1.py --pg > $O/pg_$rep.json 2> $O/pg_$rep.err || exit 1
  OMR_SIDE_QUEUES=1 timeout -k 10 120 python3 tools/round_w1.py > $O/sideq_$rep.json 2> $O/sideq_$rep.err || exit 1
  OMR_SIDE_PRIORITY=1 timeout -k 10 120 python3 tools/round_w1.py > $O/prio_$rep.json 2> $O/prio_$rep.err || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 tools/round_w1.py > $O/hwq8_$rep.json 2> $O/hwq8_$rep.err || exit 1
done
timeout -k 10 600 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
