#!/bin/bash
# Round 3, second session: one event per round for the plan's consumers (ready == planned) and no queued wait for a
# deferred round's long-fired `ready` -- the round tests, then the world-1 round under torch.distributed.run twice
# (per-round time and host time per call) and the headline line with round_world1.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03host}
mkdir -p $O
cd $R
T="python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 700 $T tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_fault.py tests/test_gpu_buckets.py \
  tests/test_gpu_round.py tests/test_gpu_msgd.py > $O/tests.log 2>&1 && \
for rep in 1 2; do
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29540+rep)) bench.py --force-dist --steps 200 --warmup 20 > $O/dist_w1_$rep.json 2> $O/dist_w1_$rep.err || exit 1
done && \
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err
