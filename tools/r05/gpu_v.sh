#!/bin/bash
# Round 5: which probe sequence leaves bench's N>1 timed rounds slow (4 IPC ranks on one GPU).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05v}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/t1_d2 29871 plain --steps 50 --warmup 10 --probe-cands thread:1,defer:2 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/d1_t2_d2 29872 plain --steps 50 --warmup 10 --probe-cands defer:1,thread:2,defer:2 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/t2_d2 29873 plain --steps 50 --warmup 10 --probe-cands thread:2,defer:2 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/t1_t2 29874 plain --steps 50 --warmup 10 --probe-cands thread:1,thread:2
