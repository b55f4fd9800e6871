#!/bin/bash
# the IPC server/client flow (one ./omr_server aggregator, two ./omr_client workers over HIP IPC,
# CHECK on) with the transport's ordering stamped (OMR_IPC_TRACE): all plain, then plain server + host-ASan clients
# (tools/r05/asan_build.sh), the mix that failed in round 5.
B=omnireduce-rdma-demo_amd/bin; A=build/asan; O=gpurun_out/${1:-r06ipc}; mkdir -p $O
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
flow() {  # $1 port, $2 tag, $3 server binary, $4 client binary, rest: client args
  P=$1; T=$2; S=$3; C=$4; shift 4
  OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $S -p $P -G 0 127.0.0.1,127.0.0.1 > $O/srv_$T.log 2>&1 & s=$!
  OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $C -X ipc -l 0 -G 0 -r 0.095 -c "$@" 127.0.0.1:$P > $O/c0_$T.log 2>&1 & c=$!
  OMR_IPC_TRACE=$O/trace_$T timeout -k 5 120 $C -X ipc -l 1 -G 0 -r 0.095 -c "$@" 127.0.0.1:$P > $O/c1_$T.log 2>&1; r1=$?
  wait $c; r0=$?; wait $s; rs=$?
  echo "$T: server rc $rs, client 0 rc $r0, client 1 rc $r1" | tee -a $O/summary.txt
  return 0
}
rm -f $O/summary.txt
flow 19911 plain $B/omr_server $B/omr_client -n 4194304 -W 2 -R 6
flow 19912 mixed $B/omr_server $A/omr_client -n 4194304 -W 2 -R 6
flow 19913 mixed2 $B/omr_server $A/omr_client -n 4194304 -W 2 -R 6
