#!/bin/bash
# Round 3, second session: plans allocating through the transport (the IPC replan fix) and its tests; where the
# world-1 round's time goes (alone, after the headline, with the host trace); the round's kernels at config-4 shapes.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03s2b}
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_ipc.py tests/test_gpu_msgd.py tests/test_cpp_dist.py > $O/tests_ipc.log 2>&1
echo "tests rc=$?" >> $O/tests_ipc.log
timeout -k 10 120 python3 tools/round_w1.py > $O/round_w1.json 2> $O/round_w1.err && \
timeout -k 10 120 python3 tools/round_w1.py --headline > $O/round_w1_headline.json 2> $O/round_w1_headline.err && \
OMR_HOST_TRACE=1 OMR_HOST_TRACE_FILE=$O/host_trace.txt timeout -k 10 120 python3 tools/round_w1.py \
  > $O/round_w1_trace.json 2> $O/round_w1_trace.err && \
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err && \
timeout -k 10 300 python3 tools/tune_round_r03.py > $O/tune_round_r03.log 2>&1 && \
timeout -k 10 300 python3 tools/tune_shard_r03.py > $O/tune_shard_r03.log 2>&1
