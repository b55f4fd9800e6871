#!/bin/bash
# Round 5: the slow timed rounds after the side-stream probe, discriminated: one side stream fixed; the probe over
# side streams with the pipeline fixed to defer; and the probe over everything (the default).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05u}
mkdir -p $O
cd $R
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_one 29861 plain --steps 50 --warmup 10 --side-streams 1 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_sides_defer 29862 plain --steps 50 --warmup 10 --dist-pipe defer || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4_auto 29863 plain --steps 50 --warmup 10
