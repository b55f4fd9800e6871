#!/bin/bash
# k_scan1f across densities at 256 MiB, B=256 (tools/tune_r02.py): the product, its no-data-store ablation and the
# pure read of its geometry, interleaved per density: how the write share of the byte mix sets the kernel's rate.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sweep
mkdir -p $O
cd $R
for d in 0.0 0.0099 0.049 0.095 0.24 0.49 1.0; do
  timeout -k 10 200 python tools/tune_r02.py --density $d --variants 0,9,14 --rounds 8 > $O/d$d.log 2>&1
done
