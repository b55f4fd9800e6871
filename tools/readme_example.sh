#!/bin/bash
# The README's CLI example on one GPU (one ./omr_server aggregator, two ./omr_client workers over the HIP IPC
# transport, the reference's default 10 + 101 rounds and its CHECK); logs under gpurun_out/readme/.
# usage (GPU box): bash tools/readme_example.sh [port]
B=omnireduce-rdma-demo_amd/bin; O=gpurun_out/readme; P=${1:-19875}; mkdir -p $O
timeout -k 5 300 $B/omr_server -p $P -G 0 127.0.0.1,127.0.0.1 > $O/srv.log 2>&1 & s=$!
timeout -k 5 300 $B/omr_client -X ipc -l 0 -G 0 -r 0.095 -c 127.0.0.1:$P > $O/c0.log 2>&1 & c=$!
timeout -k 5 300 $B/omr_client -X ipc -l 1 -G 0 -r 0.095 -c 127.0.0.1:$P > $O/c1.log 2>&1; r1=$?
wait $c; r0=$?; wait $s; rs=$?
echo "server rc $rs, client 0 rc $r0, client 1 rc $r1"
exit $(( rs || r0 || r1 ))
