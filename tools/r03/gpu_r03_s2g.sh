#!/bin/bash
# Round 3, second session: the pair-list shard sum reading its unit's length from a terminator word (one load before
# the blocks) -- parity tests, the round kernels at config-4 shapes, the round tests, PMC of the round's kernels.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2g}
mkdir -p $O
cd $R
T="python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 300 $T tests/test_gpu_pack.py > $O/tests_pack.log 2>&1 && \
timeout -k 10 300 python3 tools/tune_round_r03.py > $O/tune_round_r03.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_round.py tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_fault.py \
  > $O/tests_round.log 2>&1 && \
timeout -k 10 600 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
