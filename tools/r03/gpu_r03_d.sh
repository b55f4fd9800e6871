#!/bin/bash
# Round 3: the IPC replan failure (diagnostics with and without the fused pack), the rest of the round tests, bench
# lines and the world-1 round diagnostics, then the full-size tests.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03d}
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/ipc_replan_probe.py > $O/replan_probe.log 2>&1
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  -k replan > $O/replan_fused.log 2>&1
OMR_PACK_MOVE=1 timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_ipc.py -k replan > $O/replan_move.log 2>&1
timeout -k 10 600 python3 -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_ipc.py \
  tests/test_gpu_fault.py -k "not replan" > $O/tests.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu > $O/c2.json 2> $O/c2.err && \
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err && \
timeout -k 10 120 python3 tools/round_w1.py > $O/round_w1.json 2> $O/round_w1.err && \
timeout -k 10 120 python3 tools/round_w1.py --headline > $O/round_w1_headline.json 2> $O/round_w1_headline.err && \
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python3 tools/round_w1.py --headline > $O/round_w1_q8.json 2> $O/round_w1_q8.err && \
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  tests/test_gpu_buckets.py > $O/tests_full.log 2>&1
