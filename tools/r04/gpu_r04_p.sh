# Round 4: the pair list loading 32 records first (its tests, timing, PMC), and the world-1 round with the caller's
# stream at high priority (bench.py --caller-priority high) against normal, defer, 3 runs each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_pack.py \
  tests/test_cpp_dist.py > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/tune_round_r03.py --only "k_shard_sum" > $O/tune_round.log 2>&1
timeout -k 10 300 python3 -u tools/pmc_round.py --out $O/pmc_round_list.json --workdir $O/pmc > $O/pmc_round.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for r in 1 2 3; do
  for pr in normal high; do
    k=$((k + 1))
    MASTER_PORT=$((29760 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
      --dist-pipe defer --caller-priority $pr > $O/w1_${pr}_$r.json 2> $O/w1_${pr}_$r.err
  done
done
