#!/bin/bash
# Round 4: the round's kernels at config 4's shapes (tools/tune_round_r03.py) and their PMC HBM traffic
# (tools/pmc_round.py; FETCH_SIZE and WRITE_SIZE in separate passes).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04round}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
timeout -k 10 900 python3 -u tools/pmc_round.py --out $O/pmc_round_r04.json --workdir $O/pmc > $O/pmc_round.log 2>&1
