# Round 4: the shard sum after the 32-bit unit decode (tools/tune_shard_r04.py), then its parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 240 python -u tools/tune_shard_r04.py > $O/shard.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_round.py tests/test_cpp_dist.py -x -v -m gpu \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
