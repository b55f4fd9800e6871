#!/bin/bash
# World-1 round (bench.py --force-dist) under --dist-pipe defer and --dist-pipe thread (the progress thread),
# alternated three times to see past box drift; prints ms per round, the stage means and the host time per call.
# Lines under gpurun_out/pipe_ab/.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pipe_ab; mkdir -p $O; cd $R
port=29851
for rep in 1 2 3; do
  for pipe in defer thread; do
    port=$((port + 1))
    timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --force-dist --dist-pipe $pipe --steps 300 --warmup 20 \
      > $O/w1_${pipe}_r${rep}.json 2> $O/w1_${pipe}_r${rep}.err
    python3 - "$O/w1_${pipe}_r${rep}.json" "$pipe $rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = d["exchange"]
print(sys.argv[2], "round us", round(d["ms_per_step"] * 1e3, 1), "host us/call", round(x["host_ms_per_call"] * 1e3, 1),
      {k: round(v * 1e3, 1) for k, v in x["stages_ms"].items()})
PY
  done
done
