#!/bin/bash
# Round 3, second session: state check after the container was re-created.  The IPC replan probe, the headline bench
# line (with round_world1), then the whole -m gpu suite (no -x, so every failure shows), each under its own limit.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2a}
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/ipc_replan_probe.py > $O/replan_probe.log 2>&1
echo "replan probe rc=$?" >> $O/replan_probe.log
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err && \
timeout -k 10 950 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1
