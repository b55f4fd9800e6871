#!/bin/bash
# Round 5: the one-rank round's launch capped at 96 VGPRs (amdgpu_waves_per_eu 5): its tests, the tally scan against
# the headline (tools/tune_tally_r05.py), the world-1 round in process, and bench's N=1 line with the driver's
# arguments (headline + round_world1), and the world-1 round under torch.distributed.run.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05o}
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fault.py tests/test_gpu_round.py tests/test_cpp_dist.py tests/test_gpu_parity.py -m gpu -q -x \
  --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/tune_tally_r05.py > $O/tally.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --reps 3 --json $O/inproc.json > $O/inproc.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
