# Round 4: the non-pack worker scan with 8-wave workgroups (two per CU, OMR_SCAN_WAVES=8): parity tests with it, then
# the headline and the world-1 round, 16 against 8 waves, interleaved, 3 runs each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4u
mkdir -p $O
OMR_SCAN_WAVES=8 timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_round.py > $O/tests8.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
k=0
for r in 1 2 3; do
  for w in 16 8; do
    k=$((k + 1))
    OMR_SCAN_WAVES=$w timeout -k 10 120 python3 bench.py --no-cpu --no-round --steps 200 > $O/c2_w${w}_$r.json 2> $O/c2_w${w}_$r.err
    OMR_SCAN_WAVES=$w MASTER_PORT=$((29820 + k)) timeout -k 10 240 python3 bench.py --force-dist --no-cpu --steps 200 \
      --dist-pipe defer > $O/w1_w${w}_$r.json 2> $O/w1_w${w}_$r.err
  done
done
