#!/bin/bash
# The CLI and the round driver built with host-side AddressSanitizer (tools/r05/asan_build.sh; device code not
# instrumented): loopback rounds at one and three workers, device- and host-resident (-H), and message mode, CHECK on.
O=gpurun_out/r05oo
mkdir -p $O
B=build/asan/omr_client
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:halt_on_error=1
timeout -k 10 120 $B -L 3 -n 4194304 -r 0.095 -W 2 -R 4 -c > $O/L3.log 2>&1 || exit 1
timeout -k 10 120 $B -L 1 -n 4194304 -r 0.095 -W 2 -R 4 -c > $O/L1.log 2>&1 || exit 1
timeout -k 10 120 $B -L 3 -H -n 4194304 -r 0.3 -W 2 -R 4 -c > $O/L3H.log 2>&1 || exit 1
timeout -k 10 120 $B -L 1 -H -n 4194304 -r 0.3 -W 2 -R 4 -c > $O/L1H.log 2>&1 || exit 1
timeout -k 10 120 $B -L 3 -M -n 1048576 -r 0.3 -W 2 -R 3 -c > $O/L3M.log 2>&1 || exit 1
timeout -k 10 120 $B -L 5 -I -n 2097152 -r 0.2 -W 2 -R 3 -c > $O/L5I.log 2>&1 || exit 1
