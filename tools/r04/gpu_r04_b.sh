# Round 4, second GPU pass: the changed tests; the world-1 round (bench.py --force-dist under torch.distributed.run)
# with the row-chunk plan (default) and round 3's plan (OMR_PLAN_V1=1), alternated; one kernel trace with the host
# trace's lap times (OMR_HOST_TRACE=2, CLOCK_MONOTONIC like rocprofv3) to place the gaps between scans.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_round.py tests/test_gpu_pack.py tests/test_gpu_fault.py \
  tests/test_gpu_rccl_multi.py tests/test_bench_launch.py tests/test_gpu_buckets.py tests/test_gpu_ipc.py \
  tests/test_cpp_dist.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for rep in 1 2; do
  for v1 in 0 1; do
    OMR_PLAN_V1=$v1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29600 + rep * 2 + v1)) bench.py --force-dist --no-cpu --steps 200 \
      --warmup 20 > $O/w1_v1_${v1}_$rep.json 2> $O/w1_v1_${v1}_$rep.err
  done
done
( export MASTER_ADDR=127.0.0.1 MASTER_PORT=29613 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 OMR_HOST_TRACE=2 \
         OMR_HOST_TRACE_FILE=$O/htrace.txt
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o tl -- \
    python3 bench.py --force-dist --no-cpu --steps 100 --dist-pipe defer > $O/tl.json 2> $O/tl.err )
