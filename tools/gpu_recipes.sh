#!/bin/bash
# The GPU recipes behind DESIGN.md §5-§6, in one runner (round 6: replaces the single-use tools/r05/gpu_*.sh and
# tools/r06/gpu_*.sh, which are in git history up to commit 68ae08b).  Run on the MI355X box from the repo root:
#   gpurun --timeout 1200 -- 'bash tools/gpu_recipes.sh <recipe> <tag> [args]'
# Results go to gpurun_out/<tag>/.  Every GPU step runs under its own time limit and the steps are chained: the first
# failure ends the recipe (no retries).
#   list                      this list
#   tests TAG [files / ids]   the -m gpu suite, or only the test files / node ids given
#   final TAG                 -m gpu (slow included), smoke, bench with the driver's arguments and with its defaults,
#                             rocprofv3 --kernel-trace --stats of the default line, PMC HBM traffic of config 2
#   finalb TAG                the same without the test suite
#   bench TAG                 the other bench lines: config 3, m = 8, config 5 (N = 1), the N > 1 path at world 1
#                             (one-launch and general layouts), config 1; rocprofv3 stats of config 3; PMC of config 3
#   round TAG [filter]        the round's kernels at config 4's shapes: the launch floor (tools/tune/launch_floor.hip,
#                             built into tools/bin/ on the CPU side), timings (tools/tune_round_r03.py), then their PMC
#                             HBM traffic (tools/pmc_round.py -> pmc_round_<TAG>.json; filter: only matching cases)
#   layouts TAG               the world-1 round in its stream layouts (tools/round_inproc_r05.py: deferred, thread,
#                             after a torch group, without the queue check) and bench --world1-general with a host trace
#   w1g_trace TAG             bench --world1-general (the N > 1 path at world 1) under rocprofv3's kernel trace, deferred
#                             and with the progress thread, and its HBM bytes per round by kernel (PMC)
#   ipc_mix TAG               one ./omr_server + two ./omr_client over HIP IPC with CHECK on and OMR_IPC_TRACE: all
#                             plain, then host-AddressSanitizer clients (build/asan, tools/r05/asan_build.sh, built on
#                             the CPU side first); expected: plain passes, the mix is refused at creation
#   c5_ipc TAG                config 5's shape as 2 IPC ranks on one GPU: the staging ring against direct buckets
#   ipc_ranks TAG WORLD trace|plain [bench args]
#                             bench.py's N > 1 path as WORLD ranks sharing this GPU over HIP IPC, each a child of this
#                             shell (optionally under rocprofv3's kernel trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
recipe=${1:-list}; tag=${2:-$1}; shift 2 2>/dev/null
O=$R/gpurun_out/$tag
[ "$recipe" = list ] || mkdir -p "$O"
PORT=$((29500 + RANDOM % 400))

step() {  # step SECONDS LOGNAME cmd...: one GPU step under its own limit, stdout+stderr to $O/LOGNAME
  local secs=$1 log=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$log" 2>&1 || { echo "step $log failed (rc $?)"; tail -25 "$O/$log"; exit 1; }
}
jstep() {  # jstep SECONDS NAME cmd...: a bench line, JSON to $O/NAME.json, stderr to $O/NAME.err
  local secs=$1 name=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "bench $name failed (rc $?)"; tail -25 "$O/$name.err"; exit 1; }
}
# the N > 1 path with one rank, launched as the driver launches N > 1 (add --master-port)
DIST1=(python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1)

case "$recipe" in
list)
  sed -n '2,/^set -o pipefail/p' "$0" | sed '$d' | sed 's/^# \{0,1\}//'
  ;;
tests)
  [ $# -gt 0 ] || set -- tests  # (test files or node ids given: only those)
  step 1100 tests.log python3 -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@"
  tail -2 "$O/tests.log"
  ;;
final|finalb)
  if [ "$recipe" = final ]; then
    step 1000 gpu_tests.log python3 -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread -p no:cacheprovider
    tail -2 "$O/gpu_tests.log"
  fi
  step 300 smoke.log python3 -c "import __graft_entry__ as g; g.smoke()"
  jstep 240 c2_driver_args python3 bench.py --gpus 1 --steps 20 --warmup 5
  jstep 300 c2 python3 bench.py
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c2" -o c2 --output-format csv -- \
      python3 "$R/bench.py" --no-cpu > "$O/c2_prof.json" 2> "$O/c2_prof.err" ) || { echo "rocprofv3 failed"; exit 1; }
  step 300 pmc_c2.log python3 tools/pmc_traffic.py --out "$O/pmc_c2.json" --workdir "$O/pmc_c2"
  cat "$O/c2.json"
  ;;
bench)
  jstep 200 c3 python3 bench.py --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round
  jstep 200 m8 python3 bench.py --workers 8 --no-cpu --no-round
  jstep 200 c5 python3 bench.py --host-resident --size-mib 4096 --density 0.49 --steps 5 --warmup 1
  jstep 200 dist_w1 "${DIST1[@]}" --master-port $((PORT++)) bench.py --force-dist --steps 100 --warmup 10
  jstep 200 dist_w1_general "${DIST1[@]}" --master-port $((PORT++)) bench.py --force-dist --world1-general --no-cpu --steps 100 --warmup 10
  jstep 200 c1 python3 bench.py --size-mib 4 --density 1.0 --steps 500 --warmup 50
  ( cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o c3 --output-format csv -- \
      python3 "$R/bench.py" --size-mib 1024 --block-size 1024 --density 0.0099 --no-cpu --no-round \
      > "$O/c3_prof.json" 2> "$O/c3_prof.err" ) || { echo "rocprofv3 failed"; exit 1; }
  step 300 pmc_c3.log python3 tools/pmc_traffic.py --out "$O/pmc_c3.json" --workdir "$O/pmc_c3" -- --size-mib 1024 \
    --block-size 1024 --density 0.0099 --steps 20 --warmup 5 --no-cpu --no-round
  ;;
round)
  [ -x tools/bin/launch_floor ] && step 60 launch_floor.log tools/bin/launch_floor
  step 600 tune_round.log python3 -u tools/tune_round_r03.py --rounds 6 --reps 20 --json "$O/tune_round.json"
  step 900 pmc_round.log python3 -u tools/pmc_round.py --out "$O/pmc_round_$tag.json" --workdir "$O/pmc_work" --only "${1:-}"
  grep -v '^#' "$O/tune_round.log" | tail -25
  ;;
layouts)
  step 200 inproc.log python3 -u tools/round_inproc_r05.py --reps 2 --steps 200 --json "$O/inproc.json"
  step 200 inproc_thread.log python3 -u tools/round_inproc_r05.py --reps 2 --steps 200 --pipe thread \
    --json "$O/inproc_thread.json"
  step 200 inproc_group.log env RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((PORT++)) \
    python3 -u tools/round_inproc_r05.py --reps 2 --steps 200 --torch-group --json "$O/inproc_group.json"
  step 200 inproc_nocheck.log python3 -u tools/round_inproc_r05.py --reps 1 --steps 200 --no-queue-check \
    --json "$O/inproc_nocheck.json"
  jstep 200 w1g env OMR_HOST_TRACE=1 "${DIST1[@]}" --master-port $((PORT++)) bench.py --force-dist --world1-general --no-cpu --steps 100 --warmup 10
  jstep 200 w1g_thread env OMR_HOST_TRACE=1 "${DIST1[@]}" --master-port $((PORT++)) bench.py --force-dist --world1-general --no-cpu --dist-pipe thread \
    --side-streams 2 --steps 100 --warmup 10
  grep -h "us per round" "$O"/inproc*.log
  ;;
w1g_trace)
  for pipe in defer thread; do
    ( cd /tmp && RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((PORT++)) timeout -k 10 240 \
        rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$pipe" -o w1g -- python3 "$R/bench.py" \
        --force-dist --world1-general --no-cpu --dist-pipe $pipe --side-streams 2 --steps 100 --warmup 10 \
        > "$O/trace_$pipe.json" 2> "$O/trace_$pipe.err" ) || { echo "trace $pipe failed"; tail -20 "$O/trace_$pipe.err"; exit 1; }
  done
  step 300 pmc_w1g.log env RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((PORT++)) \
    python3 tools/pmc_traffic.py --kernel k_scan1f --also k_round_plan,k_shard_sum_list,__amd_rocclr_copyBuffer --out "$O/pmc_w1g.json" \
    --workdir "$O/pmc_w1g" -- --force-dist --world1-general --no-cpu --steps 20 --warmup 5
  ;;
ipc_mix)
  B=omnireduce-rdma-demo_amd/bin; A=build/asan
  export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
  rm -f "$O/summary.txt"
  flow() {  # flow TAG SERVER CLIENT: an aggregator and two workers, 6 rounds of 4M floats, CHECK on
    local T=$1 S=$2 C=$3 P=$((PORT++))
    OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $S -p $P -G 0 127.0.0.1,127.0.0.1 > "$O/srv_$T.log" 2>&1 & local s=$!
    OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $C -X ipc -l 0 -G 0 -r 0.095 -c -n 4194304 -W 2 -R 6 \
      127.0.0.1:$P > "$O/c0_$T.log" 2>&1 & local c=$!
    OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $C -X ipc -l 1 -G 0 -r 0.095 -c -n 4194304 -W 2 -R 6 \
      127.0.0.1:$P > "$O/c1_$T.log" 2>&1; local r1=$?
    wait $c; local r0=$?; wait $s; local rs=$?
    echo "$T: server rc $rs, client 0 rc $r0, client 1 rc $r1" | tee -a "$O/summary.txt"
    [ $rs -le 1 ] && [ $r0 -le 1 ] && [ $r1 -le 1 ] || { echo "a process of $T ended abnormally"; exit 1; }
  }
  flow plain $B/omr_server $B/omr_client
  [ -x $A/omr_client ] && flow mixed $B/omr_server $A/omr_client
  ;;
c5_ipc)
  c5() {  # c5 NAME env...: 2 ranks over HIP IPC, 4 GiB pinned per rank, -r 0.49, 256 MiB buckets
    local T=$1; shift
    env "$@" timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((PORT++)) bench.py --host-resident --dist-transport ipc --size-mib 4096 --density 0.49 --steps 3 \
      --warmup 1 > "$O/c5_$T.json" 2> "$O/c5_$T.err" || { echo "c5 $T failed"; tail -25 "$O/c5_$T.err"; exit 1; }
  }
  c5 staged OMR_RECIPE=staged
  c5 direct OMR_BUCKETS_DIRECT=1
  c5 staged2 OMR_RECIPE=staged
  c5 direct2 OMR_BUCKETS_DIRECT=1
  ;;
ipc_ranks)
  W=$1; HOW=$2; shift 2
  pids=()
  for ((r = 0; r < W; r++)); do
    if [ "$HOW" = trace ]; then
      RANK=$r LOCAL_RANK=$r WORLD_SIZE=$W LOCAL_WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/trace" -o rank$r --output-format csv -- \
        python3 "$R/bench.py" --force-dist --dist-transport ipc --no-cpu "$@" > "$O/rank$r.out" 2> "$O/rank$r.err" &
    else
      RANK=$r LOCAL_RANK=$r WORLD_SIZE=$W LOCAL_WORLD_SIZE=$W MASTER_ADDR=127.0.0.1 MASTER_PORT=$PORT \
        timeout -k 10 300 python3 "$R/bench.py" --force-dist --dist-transport ipc --no-cpu "$@" \
        > "$O/rank$r.out" 2> "$O/rank$r.err" &
    fi
    pids+=($!)
  done
  rc=0
  for p in "${pids[@]}"; do wait $p || rc=1; done
  exit $rc
  ;;
*)
  echo "unknown recipe $recipe (bash tools/gpu_recipes.sh list)"; exit 2
  ;;
esac
