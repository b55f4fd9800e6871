# Round 4, first GPU pass: the shard sum (round-3 kernel vs product), the world-1 round's kernel timeline (deferred
# pipeline; bench.py's distributed path without the torchrun launcher, kernel trace only), then the changed tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 240 python -u tools/tune_shard_r04.py > $O/shard.log 2>&1
( export MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tl_defer -o tl -- \
    python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl_defer.json 2> $O/tl_defer.err )
timeout -k 10 1000 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_round.py tests/test_gpu_fault.py \
  tests/test_gpu_rccl_multi.py tests/test_bench_launch.py tests/test_gpu_buckets.py tests/test_gpu_ipc.py \
  -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
