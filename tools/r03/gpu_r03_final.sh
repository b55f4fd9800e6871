#!/bin/bash
# Round 3 final check on one MI355X: the whole -m gpu suite, smoke, then every bench line with its profiles
# (tools/r03/gpu_bench_r03.sh).  The bench runs only if the suite ended normally (passed, or tests failed: rc 0 / 1).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03final}
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash tools/r03/gpu_bench_r03.sh ${1:-r03final}/bench
