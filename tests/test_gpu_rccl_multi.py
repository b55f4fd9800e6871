"""The product's C++ round over RCCL with one process per GPU (torch.distributed.run), as the N>1 bench runs it:
two communicators (ncclCommSplit), the mask all-gather beside the grouped send/recv exchange, zero-byte pieces
skipped on both sides, in the synchronous, asynchronous, deferred and progress-thread pipelines; every rank's outputs
checked bit for bit against the oracle (test_gpu_ipc.check_rounds).  RCCL refuses two ranks on one GPU, so these
run only where the node has the GPUs (skipped on a one-GPU box)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from omr import Layout
from test_gpu_ipc import check_rounds

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "ipc_round_worker.py")


@pytest.mark.parametrize("world,pipe,mode,B,density,rounds", [
    (2, "sync", 0, 256, 0.095, 3),
    (2, "defer", 1, 256, 0.2, 9),
    (4, "async", 0, 1024, 0.05, 5),
    (4, "defer", 0, 256, 0.3, 9),
    (8, "defer", 1, 256, 0.095, 9),
    (8, "thread", 0, 512, 0.095, 9),
])
def test_cpp_round_rccl_processes(gpu, tmp_path, world, pipe, mode, B, density, rounds):
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (RCCL refuses two ranks on one GPU)")
    L = Layout(n=2 << 20, block_size=B)
    K = min(rounds, 3)
    out = str(tmp_path / "rankRANK.npz")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--standalone", "--local-addr", "127.0.0.1", WORKER, "--transport", "rccl",
           "--floats", str(L.n), "--block", str(B), "--density", str(density), "--mode", str(mode), "--pipe", pipe,
           "--rounds", str(rounds), "--cycle", str(K), "--out", out]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    res = [np.load(out.replace("RANK", str(r))) for r in range(world)]
    check_rounds(res, L, world, B, density, mode, rounds, K)


C4_WORKER = os.path.join(HERE, "rccl_c4_worker.py")


@pytest.mark.slow
@pytest.mark.parametrize("case,extra", [
    ("c4", ["--rounds", "5"]),                 # BASELINE config 4: 8 x 256 MiB, -r 0.095, reduce-scatter + all-reduce
    ("buckets", ["--total-mib", "1024"]),      # config 5's path: pinned host, 256 MiB buckets, -r 0.49
])
def test_rccl_world8_full_size(gpu, tmp_path, case, extra):
    """The round over RCCL at BASELINE config 4's own size (256 MiB per rank, world 8, deferred rounds), every summed
    block checked against the known answer ka[count] and the chains against the oracle; and the bucketed
    pinned-host path at world 8.  Skipped below 8 GPUs."""
    world = 8
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (RCCL refuses two ranks on one GPU)")
    out = str(tmp_path / "rankRANK.txt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--standalone", "--local-addr", "127.0.0.1", C4_WORKER, "--case", case, "--out", out] + extra
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    for r in range(world):
        with open(out.replace("RANK", str(r))) as f:
            msg = f.read()
        assert msg == "ok", f"rank {r}: {msg[-3000:]}"


def test_rccl_c4_worker_fault_ends_fast(gpu, tmp_path):
    """a rank of the world-8 runs that fails must end the run at once (its error in its log, a
    non-zero exit that makes the launcher stop the other ranks), not let it run into the test's timeout.  Exercised
    at world 1 on this box: rank 0's first all-gather fails (omr_dist_inject_fault), its transport is aborted and the
    worker leaves."""
    out = str(tmp_path / "rankRANK.txt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--standalone", "--local-addr", "127.0.0.1", C4_WORKER, "--case", "c4", "--rounds", "2",
           "--fault-rank", "0", "--fault-op", "allgather", "--out", out]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
    assert p.returncode != 0, (p.stdout + p.stderr)[-3000:]
    with open(out.replace("RANK", "0")) as f:
        msg = f.read()
    assert "fault injected" in msg, msg[-3000:]
    took = float(msg.split("failed after ", 1)[1].split(" s", 1)[0])
    assert took < 30, msg[:200]
