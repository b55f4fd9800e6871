#!/bin/bash
# Round 5: side streams at the device's greatest priority (their own hardware queues): the world-1 round's layouts in
# process (three repetitions, each with fresh streams), bench's N>1 path as 4 and 8 IPC ranks, and the IPC / fault
# tests.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05bb}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --json $O/inproc.json > $O/inproc.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29941 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8 29942 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_fault.py -m gpu -q -x --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
