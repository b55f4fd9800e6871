#!/bin/bash
# Round 3, second session: the aggregation stream (an asynchronous reduce-scatter round's shard sums beside the next
# round's exchange, per-set receive buffers) -- the whole -m gpu suite, then the IPC rehearsal at world 2 / 4 with it
# on and off (host-bound on one GPU: a smoke test of the path, not a rate).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03agg}
mkdir -p $O
cd $R
timeout -k 10 700 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/tests.log 2>&1
rc=$?
echo "suite rc=$rc" >> $O/tests.log
[ $rc -le 1 ] || exit $rc
P=29701
for w in 2 4; do
  for v in on off; do
    P=$((P+1))
    if [ $v = off ]; then export OMR_AGG_STREAM=0; else unset OMR_AGG_STREAM; fi
    timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
      --master-port $P bench.py --force-dist --dist-transport ipc --no-cpu --steps 60 --warmup 10 \
      > $O/w${w}_${v}.json 2> $O/w${w}_${v}.err || exit 1
  done
done
