#!/bin/bash
# Write-request counters (rocprofv3 --pmc, one pass per counter group) for k_scan1f at config 2 and config 3:
# how the blocks' and flags' writes reach the memory side (32-byte vs 64-byte requests, stalls).
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcw
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for cfg in c2 c3; do
  if [ $cfg = c2 ]; then A="--no-cpu --steps 5 --warmup 2"; else A="--no-cpu --steps 5 --warmup 2 --size-mib 1024 --block-size 1024 --density 0.0099"; fi
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/${cfg}_a -o p --output-format csv -- python3 $R/bench.py $A > $O/${cfg}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum -d $O/${cfg}_b -o p --output-format csv -- python3 $R/bench.py $A > $O/${cfg}_b.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WR_UNCACHED_32B_sum -d $O/${cfg}_c -o p --output-format csv -- python3 $R/bench.py $A > $O/${cfg}_c.log 2>&1
done
