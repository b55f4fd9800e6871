#!/bin/bash
# Round 3: the headline bench line (with round_world1) and the whole -m gpu suite, each under its own time limit.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03a}
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
