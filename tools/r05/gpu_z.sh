#!/bin/bash
# Round 5: one side stream now destroys the idle exchange stream: the switching / IPC / C++ process tests, then bench's
# N>1 path as 8 IPC ranks with one and with two side streams fixed, and with the default probe; 4 ranks default.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05z}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_fault.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_one 29911 plain --steps 50 --warmup 10 --side-streams 1 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_two 29912 plain --steps 50 --warmup 10 --side-streams 2 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_auto 29913 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_auto 29914 plain --steps 50 --warmup 10
