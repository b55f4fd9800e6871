#!/bin/bash
# A one-rank round asked for no counts returns without waiting: the C++ round tests, the CLI loopback tests, the
# world-1 fault/RCCL tests, then config 1 through the CLI (./omr_client -L 1 -r 1.0 -n 1048576 -c) and config 2's
# loopback CLI line.
O=gpurun_out/r05gg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_cpp_dist.py \
  tests/test_gpu_fault.py -k "world1 or loopback or client or counts" > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 omnireduce-rdma-demo_amd/bin/omr_client -L 1 -r 1.0 -n 1048576 -c > $O/client_L1.log 2>&1 || exit 1
timeout -k 10 120 omnireduce-rdma-demo_amd/bin/omr_client -L 1 -r 0.095 -n 67108864 -c > $O/client_L1_c2.log 2>&1 || exit 1
