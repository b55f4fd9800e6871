#!/bin/bash
# Round 6: queue-checked side streams: the layout tests, the in-process layout study (defer, thread, torch group,
# and without the check), and bench's world-1 N>1-path line.
set -o pipefail
O=gpurun_out/${1:-r06b}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_layouts.py tests/test_gpu_ipc.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/round_inproc_r05.py --reps 2 --steps 200 --json $O/inproc.json > $O/inproc.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/round_inproc_r05.py --reps 2 --steps 200 --pipe thread --json $O/inproc_thread.json > $O/inproc_thread.log 2>&1 || exit 1
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 200 python -u tools/round_inproc_r05.py --reps 2 --steps 200 --torch-group --json $O/inproc_group.json > $O/inproc_group.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/round_inproc_r05.py --reps 1 --steps 200 --no-queue-check --json $O/inproc_nocheck.json > $O/inproc_nocheck.log 2>&1 || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --force-dist --world1-general --no-cpu --steps 100 --warmup 10 > $O/w1g.json 2> $O/w1g.err || exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --force-dist --world1-general --no-cpu --steps 20 --warmup 5 > $O/w1g_driver_args.json 2> $O/w1g_driver_args.err || exit 1
echo done
