#!/bin/bash
# Config 3 (1 GiB, B = 1024, -r 0.0099): the product launch against the study kernel in its B = 1024 form at K = 1, 2,
# 4, 8 segments per column (the product picks 2: 256 workgroups of 16 waves) and 8-wave workgroups, in place.
O=gpurun_out/r05mm
mkdir -p $O
timeout -k 10 400 python -u tools/tune_fused.py --size-mib 1024 --block-size 1024 --density 0.0099 --variants 7,18,19 \
  --ks 1,2,4,8 --rounds 10 --reps 10 > $O/c3.log 2>&1 || exit 1
