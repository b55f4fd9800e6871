#!/bin/bash
# Round 4 final check on one MI355X: the whole -m gpu suite, config 5 at its own shape, smoke (the bench lines and
# profiles are tools/r04/gpu_bench_r04.sh).  Each GPU step under its own limit; later steps run only if the suite ended
# normally (passed, or tests failed: rc 0 / 1).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04final}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "not config5_full" > $O/tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
# config 5 at its own shape (world-8 loopback, 4 GiB pinned per rank), with its wall time printed (-s)
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_buckets.py -m gpu -v -s --timeout 900 --timeout-method thread \
  -p no:cacheprovider -k config5_full > $O/tests_c5.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests_c5.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
# (the bench lines and profiles: tools/r04/gpu_bench_r04.sh, a call of its own)
