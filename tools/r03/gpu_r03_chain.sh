#!/bin/bash
# Round 3, second session: the union chain as a launch of its own in 256-thread workgroups (OMR_CHAIN_SPLIT=1) --
# round tests under the knob, then the world-1 round under torch.distributed.run with and without it, alternated.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03chain}
mkdir -p $O
cd $R
T="python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu"
OMR_CHAIN_SPLIT=1 timeout -k 10 600 $T tests/test_cpp_dist.py tests/test_gpu_ipc.py > $O/tests_split.log 2>&1 || exit 1
P=29590
for rep in 1 2; do
  for v in 0 1; do
    P=$((P+1))
    OMR_CHAIN_SPLIT=$v timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $P bench.py --force-dist --steps 200 --warmup 20 \
      > $O/w1_${v}_$rep.json 2> $O/w1_${v}_$rep.err || exit 1
  done
done
