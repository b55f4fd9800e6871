#!/bin/bash
# Round 5: bench.py as the driver runs it at N=1, and smoke, on the round's last code.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05ff}
mkdir -p $O
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_args.json 2> $O/c2_driver_args.err
