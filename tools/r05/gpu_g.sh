#!/bin/bash
# Round 5: the row-chunk plan kernel (ticketed chunks, tagged counts): parity (round/pack/fault tests), timing at
# config 4's shapes against round 3/4's form with kernel durations (rocprofv3 --kernel-trace --stats), the world-1
# round in four stream layouts, and the one-launch round's per-workgroup tally slots.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05g}
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py tests/test_gpu_fault.py -m gpu \
  -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/tune_tally_r05.py > $O/tally.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --json $O/inproc.json > $O/inproc.log 2>&1 || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/plan -o plan --output-format csv -- \
  python3 $R/tools/tune_round_r03.py --only "round plan" --rounds 4 --reps 20 --json $O/plan.json > $O/plan.log 2>&1
