# Round 4: bench.py at 16 hardware queues per process (its default now): the headline, the world-1 round (3 runs),
# and the N>1 path as 2 and 4 IPC ranks on one GPU.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 240 python3 bench.py > $O/c2.json 2> $O/c2.err
for r in 1 2 3; do
  timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $((29930 + r)) bench.py --force-dist --no-cpu --steps 200 > $O/w1_$r.json 2> $O/w1_$r.err
done
for w in 2 4; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
    --master-port $((29940 + w)) bench.py --force-dist --dist-transport ipc --no-cpu --steps 50 --warmup 10 \
    > $O/ipc_w$w.json 2> $O/ipc_w$w.err
done
