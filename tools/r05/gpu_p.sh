#!/bin/bash
# Round 5: k_scan1f's short-segment shape (small tensors): parity, config 1's bench line, and its kernel under
# rocprofv3; then the one-rank round's launch PMC (tools/pmc_traffic.py --force-dist) and a kernel trace of the round.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05p}
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_partition.py tests/test_gpu_integration.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 > $O/c1.json 2> $O/c1.err || exit 1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 300 python3 \
  tools/pmc_traffic.py --out $O/pmc_dist_w1_r05.json --workdir $O/pmc_w1 -- --force-dist --steps 20 --warmup 5 \
  > $O/pmc_w1.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c1 -o c1 --output-format csv -- \
  python3 $R/bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 --no-cpu --no-round > $O/c1_prof.json 2> $O/c1_prof.err
