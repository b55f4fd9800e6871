#!/bin/bash
# Round 5: why bench's N>1 path as 4 IPC ranks ran its timed rounds 2-3x slower than its probe: the same path with
# the side-stream probe (auto), with two side streams fixed (pipe probe only), and with no probe at all.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05t}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_fixed 29851 plain --steps 50 --warmup 10 --side-streams 2 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_pipeprobe 29852 plain --steps 50 --warmup 10 --side-streams 2 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_auto 29853 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_auto_long 29854 plain --steps 200 --warmup 10
