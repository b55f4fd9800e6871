#!/bin/bash
# Round 5: after moving the one-launch round's count publication into workgroup 0 and keeping the scan's sums on the
# hooked (N > 1 layout) world-1 path: the in-process stream-order study, the world-1 round as a torch.distributed.run
# rank, the plan kernels at config 4's shapes, then the whole -m gpu suite.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05d}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --json $O/inproc_nogroup.json > $O/inproc_nogroup.log 2>&1 || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  bench.py --force-dist --no-cpu --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err || exit 1
timeout -k 10 400 python3 -u tools/tune_round_r03.py --only "round plan" --rounds 6 --reps 20 --json $O/plan.json \
  > $O/plan.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail 15 -k "not config5_full" > $O/tests.log 2>&1
echo "suite rc=$?" >> $O/tests.log
