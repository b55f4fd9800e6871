#!/bin/bash
# Round 3 A/B on one GPU: the N>1 round rehearsed as 2 and 4 IPC processes sharing the GPU (bench.py --force-dist
# --dist-transport ipc), the fused pack (default) against the round-2 separate pack pass (OMR_PACK_MOVE=1), alternated
# twice each, and the shard sum over the plan launch's pair list (OMR_SUM_LIST=1).  Every rank's scan, pack, exchange
# and shard sum share one GPU's HBM here, so this compares the variants' total cost per round, not a multi-GPU rate.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03ab}
mkdir -p $O
cd $R
P=29601
for w in 2 4; do
  for rep in 1 2; do
    for v in fused move list; do
      P=$((P+1))
      unset OMR_PACK_MOVE OMR_SUM_LIST
      if [ $v = move ]; then export OMR_PACK_MOVE=1; fi
      if [ $v = list ]; then export OMR_SUM_LIST=1; fi
      timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
        --master-port $P bench.py --force-dist --dist-transport ipc --no-cpu --steps 60 --warmup 10 \
        > $O/w${w}_${v}_${rep}.json 2> $O/w${w}_${v}_${rep}.err || exit 1
    done
  done
done
# the loopback round tests with the pair-list shard sum (added after the final check)
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_cpp_dist.py -k sum_list > $O/tests_sum_list.log 2>&1
