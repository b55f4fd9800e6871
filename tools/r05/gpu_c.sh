#!/bin/bash
# Round 5: the world-1 round as a torch.distributed.run rank (bench --force-dist), the in-process stream-order study
# (tools/round_inproc_r05.py, with and without a torch group), the plan kernels at config 4's shapes (new vs round 3/4,
# tools/tune_round_r03.py), and the counters rocprofv3 offers (for the plan's read-request calibration).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05c}
mkdir -p $O
cd $R
(cd /tmp && timeout -k 5 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1) || true
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  bench.py --force-dist --no-cpu --steps 60 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
echo "dist_w1 rc=$?" > $O/rc.txt
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --json $O/inproc_nogroup.json > $O/inproc_nogroup.log 2>&1 || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  tools/round_inproc_r05.py --torch-group --json $O/inproc_group.json > $O/inproc_group.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/tune_round_r03.py --only "round plan" --rounds 6 --reps 20 --json $O/plan.json \
  > $O/plan.log 2>&1
