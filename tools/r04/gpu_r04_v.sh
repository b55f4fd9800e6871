# Round 4: the round's worker scan on 8-wave workgroups by default: the tests of every path that runs it, then the
# world-1 round (defer, 3 runs) and the headline (unchanged, 16 waves).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_round.py \
  tests/test_cpp_dist.py tests/test_gpu_ipc.py tests/test_gpu_buckets.py tests/test_gpu_parity.py \
  tests/test_gpu_fault.py tests/test_gpu_integration.py -k "not config5_full" > $O/tests.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for r in 1 2 3; do
  MASTER_PORT=$((29840 + r)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 --dist-pipe defer \
    > $O/w1_$r.json 2> $O/w1_$r.err
done
timeout -k 10 120 python3 bench.py --no-cpu --no-round --steps 200 > $O/c2.json 2> $O/c2.err
