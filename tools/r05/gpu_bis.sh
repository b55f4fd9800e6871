#!/bin/bash
# Round 5: bisect the 8-IPC-rank slowdown (13 ms per round at 7b6a684, 45 ms on one side stream now): bench's N>1 path
# at 8 ranks from worktrees of earlier commits (.bisect/<sha>, built in place), default arguments.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05bis}
mkdir -p $O
cd $R
port=29920
for c in 7b6a684 5c477d3 3407551; do
  port=$((port + 1))
  timeout -k 10 300 bash tools/r05/ipc_ranks_at.sh 8 $O/$c $port plain $R/.bisect/$c/bench.py --steps 50 --warmup 10 || exit 1
done
