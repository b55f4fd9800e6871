#!/bin/bash
# Bounded teardown after an abort (a peer's exchange still queued behind a 12 s kernel), then the fault, IPC and C++
# round suites on the changed transport teardown and IPC event reaper.
O=gpurun_out/r05hh
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fault.py \
  -k "destroy_bounded or one_sided" > $O/bounded.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fault.py \
  tests/test_gpu_ipc.py tests/test_cpp_dist.py > $O/suites.log 2>&1 || exit 1
