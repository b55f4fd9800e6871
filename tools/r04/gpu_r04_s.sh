# Round 4: the pair list on 8-row units (16-slot windows): its tests, then the round kernels' timings.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_pack.py \
  tests/test_cpp_dist.py -k "pack or list or sum or async" > $O/tests.log 2>&1
timeout -k 10 200 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
timeout -k 10 200 python3 -u tools/tune_shard_r04.py > $O/shard.log 2>&1
