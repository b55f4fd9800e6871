#!/bin/bash
# (Historical: k_shard_sum_pipe and OMR_SUM_PIPE were removed after this run.)
# Round 3, second session: the pipelined pair-list shard sum (k_shard_sum_pipe) and the 8-wave pack scan as defaults --
# their parity tests (and the variants behind OMR_SUM_PIPE / OMR_PACK_WAVES), the round kernels at config-4 shapes, the
# round tests, bench with the driver's arguments (round_world1 as a torch.distributed.run child), PMC of the round.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2f}
mkdir -p $O
cd $R
T="python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 300 $T tests/test_gpu_pack.py > $O/tests_pack.log 2>&1 && \
OMR_SUM_PIPE=0 timeout -k 10 300 $T tests/test_gpu_pack.py > $O/tests_pack_pipe0.log 2>&1 && \
OMR_SUM_PIPE=1 timeout -k 10 300 $T tests/test_gpu_pack.py > $O/tests_pack_pipe1.log 2>&1 && \
OMR_PACK_WAVES=16 timeout -k 10 300 $T tests/test_gpu_pack.py > $O/tests_pack_w16.log 2>&1 && \
timeout -k 10 300 python3 tools/tune_round_r03.py > $O/tune_round_r03.log 2>&1 && \
timeout -k 10 600 $T tests/test_gpu_round.py tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_fault.py \
  > $O/tests_round.log 2>&1 && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err && \
timeout -k 10 600 python3 tools/pmc_round.py --out $O/pmc_round_r03.json --workdir $O/pmc_round > $O/pmc_round.log 2>&1
