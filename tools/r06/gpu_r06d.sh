#!/bin/bash
# Round 6: the IPC mix with stamps written on abort too; bench --world1-general with the queue check on / off (A/B on
# one box) and with the host trace.
O=gpurun_out/${1:-r06d}; mkdir -p $O
bash tools/r06/gpu_ipc_trace.sh ${1:-r06d}
run() {  # $1 tag, rest: bench args
  T=$1; shift
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 300)) bench.py --force-dist --world1-general --no-cpu "$@" > $O/$T.json 2> $O/$T.err || return 1
}
run w1g_on --steps 100 --warmup 10 || exit 1
run w1g_off --queue-check off --steps 100 --warmup 10 || exit 1
run w1g_on2 --steps 100 --warmup 10 || exit 1
run w1g_off2 --queue-check off --steps 100 --warmup 10 || exit 1
run w1g_defer2 --dist-pipe defer --side-streams 2 --steps 100 --warmup 10 || exit 1
OMR_HOST_TRACE=1 run w1g_trace --dist-pipe defer --side-streams 2 --steps 100 --warmup 10 || exit 1
echo done
