#!/bin/bash
# bench's timed region closed by the barrier first over RCCL (then the synchronize): the world-1 line at the driver's
# arguments and at defaults, the distributed-path tests (RCCL world 1, IPC world 2-4), and the N=1 line.
O=gpurun_out/r05kk
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cpp_dist.py \
  -k "bench_distributed" > $O/tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 240 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
    bench.py --force-dist --no-cpu --steps 50 --warmup 10 > $O/w1_$k.json 2> $O/w1_$k.err || exit 1
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
