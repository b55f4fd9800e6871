#!/bin/bash
# The world-1 round line (bench.py --force-dist under torch.distributed.run, as round_world1's child runs it) with the
# step asking for block counts (--round-counts: the host waits for each round's publication) and without (default
# now), alternated three times; then bench's N=1 line with the driver's arguments.
O=gpurun_out/r05ii
mkdir -p $O
run() {
  timeout -k 10 240 python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
    bench.py --force-dist --no-cpu --steps 50 --warmup 10 "$@"
}
for k in 1 2 3; do
  run --round-counts > $O/w1_counts_$k.json 2> $O/w1_counts_$k.err || exit 1
  run > $O/w1_nocounts_$k.json 2> $O/w1_nocounts_$k.err || exit 1
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
