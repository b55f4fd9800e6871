# Round 4: the plan forms at config 4's shapes, then the plan parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 240 python3 -u tools/tune_round_r03.py --only "round plan" > $O/plan.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_round.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
( export MASTER_ADDR=127.0.0.1 MASTER_PORT=29613 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl -- \
    python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl.json 2> $O/tl.err )
