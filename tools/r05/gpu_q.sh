#!/bin/bash
# Round 5: two side streams again at N > 1 (plan stream + exchange stream; one at world 1): the fault / IPC / C++ round
# tests, bench's N>1 path as 2 and 4 IPC ranks on one GPU, and the world-1 round in four layouts (general = the N>1
# stream layout now).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05q}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fault.py tests/test_gpu_ipc.py tests/test_cpp_dist.py \
  tests/test_gpu_buckets.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2 29821 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29822 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --json $O/inproc.json > $O/inproc.log 2>&1
