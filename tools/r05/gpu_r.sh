#!/bin/bash
# Round 5: omr_ar_plan_set_side_streams (1 or 2 side streams, bench's N>1 probe picks on the node): the switching test
# and the multi-rank suites, bench's N>1 path as 2 and 4 IPC ranks (the probe's choice and its times), and the
# world-1 round in its layouts (one-launch; the N>1 path on two and on one side stream), with and without a torch group.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05r}
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_cpp_dist.py tests/test_gpu_fault.py tests/test_gpu_ipc.py \
  tests/test_gpu_buckets.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 2 $O/w2 29831 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 bash tools/r05/ipc_ranks.sh 4 $O/w4 29832 plain --steps 50 --warmup 10 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --json $O/inproc.json > $O/inproc.log 2>&1 || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  tools/round_inproc_r05.py --torch-group --reps 3 --json $O/inproc_group.json > $O/inproc_group.log 2>&1
