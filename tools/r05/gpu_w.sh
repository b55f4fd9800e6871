#!/bin/bash
# Round 5: does bench's N>1 path as 4 IPC ranks slow down after enough rounds, with no probe and no layout switch?
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05w}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/fixed_300 29881 plain --steps 300 --warmup 10 --side-streams 2 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/fixed_w150_s50 29882 plain --steps 50 --warmup 150 --side-streams 2 --dist-pipe defer
