#!/bin/bash
# Round 5: the fixes after gpu_a (fault tests through the world-1 hook, the plan's counts test), the world-1 round as a
# torch.distributed.run rank (bench --force-dist), and the in-process stream-order study (tools/round_inproc_r05.py).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05b}
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fault.py tests/test_gpu_round.py \
  "tests/test_gpu_rccl_multi.py::test_rccl_c4_worker_fault_ends_fast" -m gpu -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  bench.py --force-dist --no-cpu --steps 60 --warmup 10 > $O/dist_w1.json 2> $O/dist_w1.err
echo "dist_w1 rc=$?" >> $O/tests.log
timeout -k 10 300 python3 -u tools/round_inproc_r05.py --json $O/inproc_nogroup.json > $O/inproc_nogroup.log 2>&1 || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nnodes=1 --nproc-per-node 1 \
  tools/round_inproc_r05.py --torch-group --json $O/inproc_group.json > $O/inproc_group.log 2>&1
