#!/bin/bash
# Round 5: bench's N>1 path as 8 IPC ranks on one GPU with a fixed layout: one side stream, two side streams.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05y}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_one 29901 plain --steps 50 --warmup 10 --side-streams 1 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 8 $O/w8_two 29902 plain --steps 50 --warmup 10 --side-streams 2 --dist-pipe defer
