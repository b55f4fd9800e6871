#!/bin/bash
# Round 5: the plan kernel with range-checked buffer loads (parity, then timing at config 4's shapes against round
# 3/4's form), and the one-launch world-1 round's scan against the headline kernel (tools/tune_tally_r05.py).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05e}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py -m gpu -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/tune_tally_r05.py > $O/tally.log 2>&1 || exit 1
timeout -k 10 400 python3 -u tools/tune_round_r03.py --only "round plan" --rounds 6 --reps 20 --json $O/plan.json \
  > $O/plan.log 2>&1
