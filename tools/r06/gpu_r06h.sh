#!/bin/bash
# Round 6: the IPC mix traced (export / map addresses, checksums), then the round check and the changed paths' tests.
O=gpurun_out/${1:-r06h}; mkdir -p $O
bash tools/r06/gpu_ipc_trace.sh ${1:-r06h}
timeout -k 10 900 python -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py tests/test_gpu_layouts.py tests/test_gpu_ipc.py tests/test_gpu_buckets.py tests/test_cpp_dist.py tests/test_gpu_fault.py -x -v --timeout 300 --timeout-method thread -m "gpu and not slow" > $O/tests.log 2>&1; echo "tests rc=$?" >> $O/summary.txt
tail -3 $O/tests.log
