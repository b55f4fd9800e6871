#!/bin/bash
# Round 5: host-ordered side streams on the progress thread (order_after): the multi-rank suites, the world-1 round's
# layouts under defer and under thread, and bench's N>1 path as 2 and 4 IPC ranks.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05s}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_cpp_dist.py tests/test_gpu_fault.py tests/test_gpu_ipc.py \
  tests/test_gpu_buckets.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --pipe thread --json $O/inproc_thread.json > $O/inproc_thread.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --pipe defer --json $O/inproc_defer.json > $O/inproc_defer.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2 29841 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29842 plain --steps 50 --warmup 10
