#!/bin/bash
# Round 5: the IPC transport's retired events destroyed on a reaper thread (no device sync on the round's thread):
# the IPC / C++ process tests, then bench's N>1 path as 4 IPC ranks (300 timed rounds, fixed layout; and the default
# probe) and as 8 IPC ranks (the default), against the runs before (profiles/r05/side_streams/, ipc_cliff/).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05x}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_ipc.py tests/test_cpp_dist.py tests/test_gpu_msgd.py -m gpu -q -x \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_fixed_300 29891 plain --steps 300 --warmup 10 --side-streams 2 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_auto 29892 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_auto 29893 plain --steps 50 --warmup 10
