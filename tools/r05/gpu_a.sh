#!/bin/bash
# Round 5, first check of the restructured round (one side stream, the one-launch world-1 round, the single-workgroup
# plan, the compact send buffers) on one MI355X: the -m gpu suite (config 5's full shape left out), then the headline
# bench line with its world-1 round.  Each GPU step under its own limit; the bench only after a normal suite end.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05a}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --maxfail 15 -k "not config5_full" > $O/tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python3 bench.py --steps 50 --warmup 10 > $O/bench.json 2> $O/bench.err
