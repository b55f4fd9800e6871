#!/bin/bash
# Round 5's last tree: the whole -m gpu suite and smoke (the library is final5's; the CLI gained -H), then bench's
# N=1 line with the driver's arguments.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final6
mkdir -p $O
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err || exit 1
