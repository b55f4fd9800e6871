#!/bin/bash
# A one-rank group's pinned-host buckets as direct rounds (each bucket read from and its write set stored into host
# memory by one launch, no staging): the bucket tests, then config 5 at N = 1 (4 GiB, -r 0.49) with the previous
# library (build/oldpkg, staged) and the new one, alternated.
O=gpurun_out/r05ll
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_buckets.py \
  > $O/tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 300 python build/oldpkg/bench.py --host-resident --size-mib 4096 --density 0.49 > $O/c5_old_$k.json 2> $O/c5_old_$k.err || exit 1
  timeout -k 10 300 python bench.py --host-resident --size-mib 4096 --density 0.49 > $O/c5_new_$k.json 2> $O/c5_new_$k.err || exit 1
done
timeout -k 10 300 python bench.py --host-resident --size-mib 256 --density 0.095 > $O/c2_host_new.json 2> $O/c2_host_new.err || exit 1
timeout -k 10 300 python build/oldpkg/bench.py --host-resident --size-mib 256 --density 0.095 > $O/c2_host_old.json 2> $O/c2_host_old.err || exit 1
