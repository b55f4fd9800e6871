#!/bin/bash
# Round 6: the IPC mix (expected: the canary check refuses the group at creation, naming the offset), the changed
# paths' tests (round check, layouts, IPC, buckets, C++ processes, faults), then config 5's shape as 2 IPC ranks on
# one GPU: rounds on the mapped pinned buckets (round 6 default) against the staging ring.
O=gpurun_out/${1:-r06i}; mkdir -p $O
bash tools/r06/gpu_ipc_trace.sh ${1:-r06i}
timeout -k 10 900 python -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py tests/test_gpu_layouts.py tests/test_gpu_ipc.py tests/test_gpu_buckets.py tests/test_cpp_dist.py tests/test_gpu_fault.py -x -v --timeout 300 --timeout-method thread -m "gpu and not slow" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
c5() {  # $1 tag, rest: env
  T=$1; shift
  env "$@" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) bench.py --host-resident --dist-transport ipc --size-mib 4096 --density 0.49 --steps 3 --warmup 1 > $O/c5_$T.json 2> $O/c5_$T.err || return 1
}
c5 direct OMR_X=1 || exit 1
c5 staged OMR_BUCKETS_STAGED=1 || exit 1
c5 direct2 OMR_X=1 || exit 1
c5 staged2 OMR_BUCKETS_STAGED=1 || exit 1
echo done
