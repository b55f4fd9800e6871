#!/bin/bash
# Round 5: the pair list's workgroups spread over the XCDs by row group (xcd_spread): parity (round / pack tests),
# the plan launch's time at config 4's shapes, and its HBM traffic with the request-size counters.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05m}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py -m gpu -q -x --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/tune_round_r03.py --only "round plan" --rounds 6 --reps 20 > $O/plan.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/pmc_round.py --only "round plan as the round calls it" --out $O/pmc_plan.json \
  --workdir $O/pmc > $O/pmc.log 2>&1
