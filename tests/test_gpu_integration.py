"""INTEGRATION.md's worker recipe compiled as C++ and run as the reference runs a worker (tests/integration/
worker_partition.cpp): the gradient in a posix_memalign'd host region filled by the reference generator itself
(srand(id+1), glibc rand(), client.cc:396-421), NUM_THREADS std::threads each on its own HIP stream calling
omr_scan_partition_f32 on its partition (client.cc:168, :384-392), every next offset compared with the oracle's
find_next_nonzero_block (client.cc:19-31) as client.cc:94/:203 call it, every flag with the bitmap, and the in-place
aggregated blocks bit for bit."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "integration", "worker_partition")


@pytest.mark.parametrize("n,B,r,wid", [(16 << 20, 256, 0.095, 0), (16 << 20, 1024, 0.0099, 3), (8 << 20, 512, 0.49, 1),
                                      (64 << 20, 256, 0.095, 0)])  # the last: config 2 (256 MiB)
def test_integration_worker_partition(gpu, n, B, r, wid):
    assert os.path.exists(BIN), "build it: make -C tests/integration (done by __graft_entry__.build())"
    res = subprocess.run([BIN, "-n", str(n), "-b", str(B), "-r", str(r), "-i", str(wid)], capture_output=True,
                         text=True, timeout=180)
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.count("next mismatches 0, flag mismatches 0") == 2 and "out equal" in res.stdout, res.stdout
