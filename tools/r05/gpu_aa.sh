#!/bin/bash
# Round 5: IPC plans default to one side stream beyond 4 ranks: the IPC / C++ process / fault tests, then bench's
# N>1 path as 2, 4 and 8 IPC ranks on one GPU with its defaults.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05aa}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ipc.py tests/test_cpp_dist.py tests/test_gpu_fault.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2 29931 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29932 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8 29933 plain --steps 50 --warmup 10
