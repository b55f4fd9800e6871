#!/bin/bash
# Round 5, last code: the whole -m gpu suite and smoke, then the bench lines (the driver's N=1 arguments; the default
# run with cpu_baseline and round_world1; configs 1, 3, m = 8; the world-1 round as its own line), and the headline's
# rocprofv3 kernel stats.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final2}
mkdir -p $O
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
timeout -k 10 300 python3 bench.py > $O/c2.json 2> $O/c2.err || exit 1
timeout -k 10 300 python3 bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50 > $O/c1.json 2> $O/c1.err || exit 1
timeout -k 10 200 python3 bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 200 python3 bench.py --workers 8 --no-cpu --no-round > $O/m8.json 2> $O/m8.err || exit 1
timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --force-dist --steps 100 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o c2 --output-format csv -- \
  python3 $R/bench.py --no-cpu --no-round > $O/c2_prof.json 2> $O/c2_prof.err
