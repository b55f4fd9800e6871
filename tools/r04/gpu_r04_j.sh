# Round 4: 16-row shard-sum units; the world-1 round with 3 or 4 round sets (OMR_ROUND_SETS), defer and thread.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 300 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
timeout -k 10 240 python3 -u tools/tune_shard_r04.py > $O/shard.log 2>&1
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_pack.py \
  tests/test_gpu_round.py tests/test_gpu_ipc.py tests/test_cpp_dist.py tests/test_gpu_fault.py > $O/tests.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for r in 1 2 3; do
  for sets in 3 4; do
    for pipe in defer thread; do
      MASTER_PORT=$((29700 + r * 4 + sets)) OMR_ROUND_SETS=$sets timeout -k 10 240 python3 bench.py --force-dist \
        --no-cpu --steps 200 --dist-pipe $pipe > $O/w1_s${sets}_${pipe}_$r.json 2> $O/w1_s${sets}_${pipe}_$r.err
    done
  done
done
