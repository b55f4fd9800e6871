#!/bin/bash
# Round 5: the row-chunk plan's study variants at config 4's shapes (tools/tune_plan_v5.py) under rocprofv3's
# kernel trace (per-variant kernel durations).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05j}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o v5 --output-format csv -- \
  python3 $R/tools/tune_plan_v5.py > $O/v5.log 2>&1
