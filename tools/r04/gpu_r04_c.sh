# Round 4, third GPU pass: first-load latency at kernel start (the shard sum's index phase); the N>1 round rehearsed
# as 2 and 4 IPC processes on this GPU (the pack scan, exchanges and shard sums of every rank share its HBM) with the
# row-chunk plan (OMR_PLAN_V1=0) and round 3's plan (1), alternated twice.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 240 python3 -u tools/tune_lat_r04.py > $O/lat.log 2>&1
P=29701
for w in 2 4; do
  for rep in 1 2; do
    for v1 in 0 1; do
      P=$((P+1))
      OMR_PLAN_V1=$v1 timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w \
        --master-addr 127.0.0.1 --master-port $P bench.py --force-dist --dist-transport ipc --no-cpu --steps 60 \
        --warmup 10 > $O/w${w}_v1_${v1}_${rep}.json 2> $O/w${w}_v1_${v1}_${rep}.err
    done
  done
done
