#!/bin/bash
# Round 5 (an experiment build, not kept: its host code read the cap from OMR_EXP_LIST_WGS): the plan launch's
# pair-list workgroup count (512 / 256 / 128 / 64): the plan alone at
# config 4's shapes and the multi-rank path at world 1 in bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05ee}
mkdir -p $O
cd $R
for n in 512 128 256 64; do
  OMR_EXP_LIST_WGS=$n timeout -k 10 300 python3 -u tools/tune_round_r03.py --only "round plan as the round calls it (pair" \
    --rounds 6 --reps 20 > $O/plan_$n.log 2>&1 || exit 1
  OMR_EXP_LIST_WGS=$n timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29550 + n % 97)) bench.py --force-dist --world1-general --dist-pipe defer --side-streams 2 --steps 100 \
    --warmup 10 > $O/w1g_$n.json 2> $O/w1g_$n.err || exit 1
done
