#!/bin/bash
# Round 5: the N>1 round's pipeline in a multi-rank kernel timeline: bench's N>1 path as 2 IPC ranks on one GPU, two
# side streams, deferred, one rocprofv3 kernel trace per rank (queue ids: the caller's scans against the plan and
# exchange streams' kernels and copies).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05cc}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2_trace 29951 trace --steps 30 --warmup 10 --side-streams 2 --dist-pipe defer
