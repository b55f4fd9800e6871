# Round 4: the shard sum forms (tools/tune_shard_r04.py) and their parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 240 python -u tools/tune_shard_r04.py > $O/shard.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_round.py -x -v -m gpu \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
