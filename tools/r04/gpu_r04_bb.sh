# Round 4: OMR_ROUND_SHIFT=1 (a deferred round's first half issued by the next call, after its scan): the round tests
# with it, then the world-1 round with and without it in the fast configuration (bench child) and in the in-process
# configurations that ran 2x slower (tools/round_inproc_r04.py --comm-first, with / without a torch group).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4bb
mkdir -p $O
OMR_ROUND_SHIFT=1 timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread \
  tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_round.py tests/test_gpu_fault.py > $O/tests.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for r in 1 2; do
  for sh in 0 1; do
    k=$((k + 1))
    OMR_ROUND_SHIFT=$sh MASTER_PORT=$((29950 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu \
      --steps 200 --dist-pipe defer > $O/w1_s${sh}_$r.json 2> $O/w1_s${sh}_$r.err
  done
done
for sh in 0 1; do
  k=$((k + 1))
  OMR_ROUND_SHIFT=$sh timeout -k 10 150 python3 -u tools/round_inproc_r04.py --comm-first > $O/nogroup_s$sh.log 2>&1
  OMR_ROUND_SHIFT=$sh MASTER_PORT=$((29950 + k)) timeout -k 10 150 python3 -u tools/round_inproc_r04.py \
    --comm-first --torch-group > $O/group_s$sh.log 2>&1
done
