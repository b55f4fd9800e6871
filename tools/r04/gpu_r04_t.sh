# Round 4: bench.py's N>1 path rehearsed as 2, 4 and 8 ranks on one GPU over HIP IPC with the round-4 defaults
# (pair-list shard sum, four round sets): not scaling figures, a check that the N>1 lines run end to end.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4t
mkdir -p $O
for w in 2 4 8; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29800 + w)) bench.py --force-dist --dist-transport ipc --no-cpu --steps 50 --warmup 10 \
    > $O/ipc_w$w.json 2> $O/ipc_w$w.err
done
