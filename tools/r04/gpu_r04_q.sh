# Round 4: rounds without a requested union chain skip it in the plan launch: the round tests, then the world-1
# round (defer and thread, 3 runs each) and its kernel trace.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_cpp_dist.py \
  tests/test_gpu_ipc.py tests/test_gpu_round.py tests/test_gpu_fault.py tests/test_gpu_buckets.py \
  tests/test_gpu_rccl_multi.py -k "not config5_full" > $O/tests.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for r in 1 2 3; do
  for pipe in defer thread; do
    k=$((k + 1))
    MASTER_PORT=$((29780 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
      --dist-pipe $pipe > $O/w1_${pipe}_$r.json 2> $O/w1_${pipe}_$r.err
  done
done
MASTER_PORT=29799 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tl -o tl -- \
  python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl.json 2> $O/tl.err
