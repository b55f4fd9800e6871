#!/bin/bash
# bench.py's N>1 path as 2, 4 and 8 IPC ranks on one GPU with the round's last code (a rehearsal: the ranks share one
# GPU and its hardware queues).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ipc_final
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2 29941 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29942 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8 29943 plain --steps 50 --warmup 10
