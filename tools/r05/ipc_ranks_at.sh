#!/bin/bash
# Start bench.py's N>1 path as $1 ranks on this box's GPU over HIP IPC (a rehearsal: the ranks share one GPU), each rank
# a child of this shell (no launcher process in between), optionally each under rocprofv3's kernel trace.
# usage: ipc_ranks_at.sh WORLD OUTDIR PORT trace|plain BENCH_PY [bench args...]
W=$1; O=$2; PORT=$3; HOW=$4; BENCH=$5; shift 5
mkdir -p $O
pids=()
for ((r = 0; r < W; r++)); do
  if [ "$HOW" = trace ]; then
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$W LOCAL_WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
      rocprofv3 --kernel-trace -d $O/trace -o rank$r --output-format csv -- \
      python3 $BENCH --force-dist --dist-transport ipc --no-cpu "$@" > $O/rank$r.out 2> $O/rank$r.err &
  else
    RANK=$r LOCAL_RANK=$r WORLD_SIZE=$W LOCAL_WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
      python3 $BENCH --force-dist --dist-transport ipc --no-cpu "$@" > $O/rank$r.out 2> $O/rank$r.err &
  fi
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
