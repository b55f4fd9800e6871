#!/bin/bash
# The IPC server/client flow (one ./omr_server aggregator, two ./omr_client workers over HIP IPC, CHECK on) with the
# normal builds and with host-side AddressSanitizer builds (tools/r05/asan_build.sh), mixed and matched.
B=omnireduce-rdma-demo_amd/bin; A=build/asan; O=gpurun_out/r05pp; mkdir -p $O
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1
flow() {  # $1 port, $2 tag, $3 server binary, $4 client binary, rest: client args
  P=$1; T=$2; S=$3; C=$4; shift 4
  timeout -k 5 300 $S -p $P -G 0 127.0.0.1,127.0.0.1 > $O/srv_$T.log 2>&1 & s=$!
  timeout -k 5 300 $C -X ipc -l 0 -G 0 -r 0.095 -c "$@" 127.0.0.1:$P > $O/c0_$T.log 2>&1 & c=$!
  timeout -k 5 300 $C -X ipc -l 1 -G 0 -r 0.095 -c "$@" 127.0.0.1:$P > $O/c1_$T.log 2>&1; r1=$?
  wait $c; r0=$?; wait $s; rs=$?
  echo "$T: server rc $rs, client 0 rc $r0, client 1 rc $r1" | tee -a $O/summary.txt
  return 0
}
rm -f $O/summary.txt
flow 19904 plainsrv_asanexe_plainlib $B/omr_server build/asan_exe/omr_client -n 4194304
flow 19905 mixed_again $B/omr_server $A/omr_client -n 4194304
