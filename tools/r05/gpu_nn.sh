#!/bin/bash
# ./omr_client -H (the tensor in pinned host memory, as the reference's registered res->buf): the CLI tests, then
# config 1 and config 2 through the CLI with -H, one worker on loopback, CHECK on.
O=gpurun_out/r05nn
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cpp_dist.py \
  -k "client" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 omnireduce-rdma-demo_amd/bin/omr_client -L 1 -H -r 1.0 -n 1048576 -c > $O/client_L1_H_c1.log 2>&1 || exit 1
timeout -k 10 120 omnireduce-rdma-demo_amd/bin/omr_client -L 1 -H -r 0.095 -n 67108864 -c > $O/client_L1_H_c2.log 2>&1 || exit 1
