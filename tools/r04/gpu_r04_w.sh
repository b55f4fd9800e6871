# Round 4: the round's worker scan on 4-wave workgroups (OMR_SCAN_WAVES=4) against the 8-wave default: parity tests
# with 4, then the world-1 round, interleaved, 3 runs each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4w
mkdir -p $O
OMR_SCAN_WAVES=4 timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_round.py > $O/tests4.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for r in 1 2 3; do
  for w in 8 4; do
    k=$((k + 1))
    OMR_SCAN_WAVES=$w MASTER_PORT=$((29860 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
      --dist-pipe defer > $O/w1_w${w}_$r.json 2> $O/w1_w${w}_$r.err
  done
done
