#!/bin/bash
# Host-side AddressSanitizer builds of the round driver and the CLI (device code is not instrumented:
# -fno-gpu-sanitize), into build/asan/: libomr_dist.so and omr_client, linked against the normal libomr.so.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/omnireduce-rdma-demo_amd
O=$R/build/asan
mkdir -p $O
F="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -fsanitize=address -fno-gpu-sanitize -fno-omit-frame-pointer -I$R/include"
/opt/rocm/bin/hipcc $F -shared -o $O/libomr_dist.so $P/csrc/omr_dist.hip -L$P/omr -lomr -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,$P/omr -Wl,-rpath,/opt/rocm/lib
/opt/rocm/bin/hipcc $F -o $O/omr_client $P/host/omr_client.cpp -L$O -lomr_dist -L$P/omr -lomr -lpthread \
  -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$P/omr -Wl,-rpath,/opt/rocm/lib
echo built $O
/opt/rocm/bin/hipcc $F -o $O/omr_server $P/host/omr_server.cpp -L$O -lomr_dist -L$P/omr -lomr -lpthread \
  -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$P/omr -Wl,-rpath,/opt/rocm/lib
echo built $O/omr_server
