#!/bin/bash
# k_scan1f's block-store cache policy in place (the headline) and out of place with one output per input set (the
# world-1 round's shape): k_scanm's out-of-place sums preferred nt stores by 7 %.
O=gpurun_out/r05jj
mkdir -p $O
timeout -k 10 300 python -u tools/tune_fused.py --variants 11,12,13,14,15,16,17 --ks 1 --rounds 20 > $O/inplace.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/tune_fused.py --variants 11,12,13,14,15,16,17 --ks 1 --rounds 20 --out-of-place \
  > $O/outofplace.log 2>&1 || exit 1
