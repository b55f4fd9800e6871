#!/bin/bash
# k_scanm round-2 evidence on one MI355X: parity, the side-by-side study, bench m=8 under rocprofv3 (kernel trace
# + stats), HBM traffic (FETCH_SIZE / WRITE_SIZE passes).  Every GPU step under its own time limit, chained with &&.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/scanm
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  "tests/test_gpu_fullsize.py::test_c4_scanm_m8" > $O/tests.log 2>&1
timeout -k 10 200 python -u tools/tune_scanm_r02.py --sets 4 --rounds 12 > $O/tune.log 2>&1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o m8 --output-format csv -- \
  python3 $R/bench.py --workers 8 --steps 40 --warmup 5 --no-cpu > $O/bench_m8_prof.log 2>&1
timeout -k 10 300 python3 $R/tools/pmc_traffic.py --kernel k_scanm --out $O/pmc_m8_r02.json --workdir $O/pmc -- \
  --workers 8 --steps 20 --warmup 5 --no-cpu > $O/pmc.log 2>&1
cd $R
timeout -k 10 200 python3 bench.py --workers 8 --steps 40 --warmup 5 --no-cpu --pmc $O/pmc_m8_r02.json > $O/bench_m8.log 2>&1
