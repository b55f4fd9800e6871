# Round 4: the pair list on 16-row units after the geometry fix: its tests first, then the kernels' timings, the
# round-gap study, then the final test check.  Each step stops the script on failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests/test_gpu_pack.py \
  > $O/tests_pack.log 2>&1
timeout -k 10 200 python3 -u tools/tune_round_r03.py > $O/tune_round.log 2>&1
timeout -k 10 200 python3 -u tools/tune_shard_r04.py > $O/shard.log 2>&1
timeout -k 10 200 python3 -u tools/round_gap_r04.py > $O/gap.log 2>&1
bash tools/r04/gpu_r04_final.sh r04final
