#!/bin/bash
# Round 3, second session: where a world-1 round's host time goes in the N>1 bench's own set-up (OMR_HOST_TRACE=1,
# per-step host time summed over the rounds and printed at plan destroy), deferred and with the progress thread.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03htrace}
mkdir -p $O
cd $R
for pipe in defer thread; do
  OMR_HOST_TRACE=1 timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --force-dist --dist-pipe $pipe --steps 200 --warmup 20 \
    > $O/w1_$pipe.json 2> $O/w1_$pipe.err || exit 1
done
