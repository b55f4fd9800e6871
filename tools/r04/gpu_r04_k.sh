# Round 4: is the world-1 round's 5-11 us gap between scans a hardware-queue share?  The round at 4 (the box default)
# and 8 hardware queues per process (GPU_MAX_HW_QUEUES), defer and thread, then a kernel trace at 8.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4k
mkdir -p $O
export MASTER_ADDR=127.0.0.1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 OMR_ROUND_SETS=4
for r in 1 2; do
  for q in 4 8; do
    for pipe in defer thread; do
      MASTER_PORT=$((29720 + r * 10 + q)) GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python3 bench.py --force-dist \
        --no-cpu --steps 200 --dist-pipe $pipe > $O/w1_q${q}_${pipe}_$r.json 2> $O/w1_q${q}_${pipe}_$r.err
    done
  done
done
export GPU_MAX_HW_QUEUES=8 MASTER_PORT=29750 OMR_HOST_TRACE=2 OMR_HOST_TRACE_FILE=$GRAFT_REPO_ROOT/$O/htrace_q8.txt
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl -- \
  python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl.json 2> $O/tl.err
