#!/bin/bash
# Round 3, second session: the shard sum's pair list built by the plan launch -- its parity tests, the round tests that
# take it (loopback, IPC processes, fault injection), the round kernels at config-4 shapes; then bench (headline +
# round_world1 behind a one-rank torch group), kernel traces of the world-1 round with / without that group, and PMC.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2e}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_pack.py > $O/tests_pack.log 2>&1 && \
OMR_PACK_WAVES=16 timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  -m gpu tests/test_gpu_pack.py > $O/tests_pack_w16.log 2>&1 && \
timeout -k 10 300 python3 tools/tune_round_r03.py > $O/tune_round_r03.log 2>&1 && \
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_round.py tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_fault.py > $O/tests_round.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err && \
cd /tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_group -o w1 --output-format csv -- \
  python3 $R/tools/round_w1.py --steps 40 > $O/trace_group.json 2> $O/trace_group.err && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_nogroup -o w1 --output-format csv -- \
  python3 $R/tools/round_w1.py --steps 40 --no-group > $O/trace_nogroup.json 2> $O/trace_nogroup.err && \
cd $R && \
timeout -k 10 600 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
