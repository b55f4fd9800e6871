#!/bin/bash
# World-1 round (bench.py --force-dist, deferred pipeline) with the round events recorded with (OMR_EVENT_SYSFENCE=1)
# and without a system-scope fence, alternated to see past box drift.  Lines under gpurun_out/sysfence/.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sysfence; mkdir -p $O; cd $R
port=29711
for rep in 1 2 3; do
  for pr in 0 1; do
    port=$((port + 1))
    OMR_EVENT_SYSFENCE=$pr timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $port bench.py --force-dist --steps 200 --warmup 20 \
      > $O/w1_p${pr}_r${rep}.json 2> $O/w1_p${pr}_r${rep}.err
    echo "prio $pr rep $rep: $(python3 -c "import json,sys; d=json.loads(open('$O/w1_p${pr}_r${rep}.json').read().strip().splitlines()[-1]); print(d['ms_per_step']*1e3, 'us/round', d['roofline']['kernel_ms']*1e3, 'us scan')")"
  done
done
