# Round 4: the scan's completion signal (no event between the caller's back-to-back scans): its tests, the round
# tests around it, the shard sum's store policies (stamped copies), then the world-1 round A/B (OMR_SCAN_SIGNAL=0 / 1, interleaved) and a kernel trace with it on.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h
mkdir -p $O
T="python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_pack.py -k signal > $O/signal.log 2>&1
timeout -k 10 240 python3 -u tools/tune_shard_r04.py > $O/shard_pol.log 2>&1
timeout -k 10 900 $T tests/test_gpu_round.py tests/test_gpu_fault.py tests/test_gpu_ipc.py tests/test_cpp_dist.py \
  tests/test_gpu_buckets.py -k "not config5_full" > $O/tests.log 2>&1
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
for r in 1 2 3; do
  for s in 0 1; do
    for pipe in defer thread; do
      MASTER_PORT=$((29620 + r * 4 + s * 2)) OMR_SCAN_SIGNAL=$s timeout -k 10 240 python3 bench.py --force-dist \
        --no-cpu --steps 200 --dist-pipe $pipe > $O/ab_s${s}_${pipe}_$r.json 2> $O/ab_s${s}_${pipe}_$r.err
    done
  done
done
MASTER_PORT=29650 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl -- \
  python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl.json 2> $O/tl.err
