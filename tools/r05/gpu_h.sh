#!/bin/bash
# Round 5: the 8-rank IPC rehearsal's cliff (31.5 ms per round at 8 ranks on one GPU against
# 1.36 ms at 4).  One kernel trace of 8 ranks (rocprofv3, one file per rank: queue ids, start/end per kernel), then
# the same 8 ranks untraced with GPU_MAX_HW_QUEUES=2 (16 hardware queues over the processes instead of 32+), and 4
# ranks untraced with the default, for the per-round figures beside it.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05h}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_trace 29811 trace --steps 20 --warmup 5 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29812 plain --steps 50 --warmup 10 || exit 1
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_hwq2 29813 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8 29814 plain --steps 50 --warmup 10
