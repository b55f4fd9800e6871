#!/bin/bash
# Round 5: kernel durations (rocprofv3 --kernel-trace --stats) of the plan kernels (round 5's single workgroup vs round
# 3/4's per-array workgroups) and of the one-launch round's tally scan vs the headline kernel, to tell kernel time from
# launch gaps in the event-timed loops.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05f}
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plan -o plan --output-format csv -- \
  python3 $R/tools/tune_round_r03.py --only "round plan, no chain" --rounds 3 --reps 10 > $O/plan.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tally -o tally --output-format csv -- \
  python3 $R/tools/tune_tally_r05.py > $O/tally.log 2>&1
