# Round 4: the shard sum's phases (stamped copy of the product kernel, tools/make_shard_r04.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 240 python -u tools/tune_shard_r04.py > $O/shard.log 2>&1
