# Round 4: bench.py's N>1 path as 2 and 4 IPC ranks on one GPU with two side streams (the N>1 default) and with one
# (OMR_ONE_SIDE_STREAM=1), interleaved, 2 runs each: does the world-1 fix carry to N>1?
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4ee
mkdir -p $O
k=0
for r in 1 2; do
  for w in 2 4; do
    for one in 0 1; do
      k=$((k + 1))
      OMR_ONE_SIDE_STREAM=$one timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w \
        --master-addr 127.0.0.1 --master-port $((29980 + k)) bench.py --force-dist --dist-transport ipc --no-cpu \
        --steps 50 --warmup 10 > $O/ipc_w${w}_o${one}_$r.json 2> $O/ipc_w${w}_o${one}_$r.err
    done
  done
done
