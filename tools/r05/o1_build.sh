#!/bin/bash
# -O1 -g builds (no sanitizer) of the round driver, the CLI and the server, into build/o1/: to tell an optimisation-
# level effect from a sanitizer one when builds are mixed.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/omnireduce-rdma-demo_amd
O=$R/build/o1
mkdir -p $O
F="--offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -I$R/include"
/opt/rocm/bin/hipcc $F -shared -o $O/libomr_dist.so $P/csrc/omr_dist.hip -L$P/omr -lomr -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,$P/omr -Wl,-rpath,/opt/rocm/lib
for b in omr_client omr_server; do
  /opt/rocm/bin/hipcc $F -o $O/$b $P/host/$b.cpp -L$O -lomr_dist -L$P/omr -lomr -lpthread \
    -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$P/omr -Wl,-rpath,/opt/rocm/lib
done
echo built $O
