#!/bin/bash
# Round 3, second session: the plan launch in 256-thread workgroups (OMR_PLAN_THREADS=256, so they can share a CU with a
# running scan workgroup) -- plan / pack / round tests under the knob, then the world-1 round under
# torch.distributed.run with and without it, alternated twice, and the round kernels at config-4 shapes with it.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03plan}
mkdir -p $O
cd $R
T="python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu"
OMR_PLAN_THREADS=256 timeout -k 10 600 $T tests/test_gpu_round.py tests/test_gpu_pack.py tests/test_cpp_dist.py \
  > $O/tests_256.log 2>&1 || exit 1
P=29580
for rep in 1 2; do
  for v in 1024 256; do
    P=$((P+1))
    OMR_PLAN_THREADS=$v timeout -k 10 200 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $P bench.py --force-dist --steps 200 --warmup 20 \
      > $O/w1_${v}_$rep.json 2> $O/w1_${v}_$rep.err || exit 1
  done
done
OMR_PLAN_THREADS=256 timeout -k 10 300 python3 tools/tune_round_r03.py > $O/tune_round_r03_256.log 2>&1
