# Round 4: write-through (kStoreAux) block stores in the fused pack, the shard sums and k_move: the round's kernels at
# config 4's shapes, the shard sum's stamped copies, then the tests that cover those kernels.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 300 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
timeout -k 10 240 python3 -u tools/tune_shard_r04.py > $O/shard.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_pack.py \
  tests/test_gpu_round.py tests/test_gpu_parity.py tests/test_gpu_partition.py > $O/tests.log 2>&1
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fault.py \
  tests/test_gpu_rccl_multi.py > $O/tests_rccl.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for r in 1 2 3; do
  for pipe in defer thread; do
    MASTER_PORT=$((29660 + r * 2)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
      --dist-pipe $pipe > $O/w1_${pipe}_$r.json 2> $O/w1_${pipe}_$r.err
  done
done
MASTER_PORT=29690 OMR_HOST_TRACE=1 timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 100 \
  --dist-pipe defer > $O/htrace.json 2> $O/htrace.err
