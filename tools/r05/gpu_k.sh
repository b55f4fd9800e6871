#!/bin/bash
# Round 5: the full -m gpu suite after the row-chunk plan, then HBM traffic of the round's kernels at config 4's shapes
# (tools/pmc_round.py: FETCH_SIZE / WRITE_SIZE passes and the read-request-size counters, one pass each).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05k}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python3 tools/pmc_round.py --out $O/pmc_round_r05.json --workdir $O/pmc_round > $O/pmc.log 2>&1
