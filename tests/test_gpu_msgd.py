"""The message-level round between separate worker and aggregator PROCESSES (omr_msgd_*, HIP-IPC transport on the
one GPU): every worker message and every aggregator reply, byte for byte, equals the oracle's literal restatement of
the per-slot state machines (orc_msg_simulate: client.cc:32-205, server.cc:13-199), the slots sharded over the
aggregators by gs % n (common.cc:381-383), and every worker ends with the reference CHECK's known answer (the
rank-order sums, client.cc:449-465)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from omr import Layout, cdist

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ipc_msgd_worker.py")


@pytest.mark.parametrize("m,naggs,B,density", [(2, 1, 256, 0.2), (3, 2, 256, 0.3), (2, 3, 1024, 0.1),
                                               (3, 0, 512, 0.2)])
def test_msgd_processes_vs_state_machines(gpu, tmp_path, m, naggs, B, density):
    n = 1 << 20
    world = m + naggs
    uid = cdist.ipc_unique_id().hex()
    procs = []
    for r in range(world):
        cmd = [sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--workers", str(m), "--uid", uid,
               "--n", str(n), "--block", str(B), "--density", str(density), "--out", str(tmp_path / f"r{r}.npz")]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("a msgd rank hung")
    for r, p in enumerate(procs):
        assert p.returncode == 0, logs[r]
    res = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    L = Layout(n=n, block_size=B)
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B) for w in range(m)]
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    ref = oracle.msg_simulate(bufs, flags, n, B, L.num_lanes, L.num_threads)
    G = L.num_threads * 16
    A = naggs if naggs else m  # co-located: every worker also aggregates
    rounds = ref["rounds"]
    dense = np.zeros(n, dtype=np.float32)
    oracle.block_sum(bufs, n, B, L.num_lanes, L.num_threads, oracle.union_flags(flags), dense)
    for w in range(m):
        z = res[w]
        assert (z["rounds"] == rounds).all()
        assert (z["out"].view(np.uint32) == ref["outs"][w].view(np.uint32)).all(), f"worker {w} result"
        assert (z["out"].view(np.uint32) == dense.view(np.uint32)).all(), f"worker {w} known answer"
        for gs in range(G):
            for rr in range(int(rounds[gs])):
                imm = int(ref["wimm"][w, gs, rr])
                assert int(z["imm"][gs, rr]) == imm, (w, gs, rr)
                ln = imm >> 16
                assert z["msg"][gs, rr, :ln * B + ln].tobytes() == ref["wmsg"][w, gs, rr, :ln * B + ln].tobytes()
                rimm = int(ref["rimm"][gs, rr])
                assert int(z["rimm"][gs, rr]) == rimm, (w, gs, rr, "reply")
                ln = rimm >> 16
                assert z["reply"][gs, rr, :ln * B + ln].tobytes() == ref["rmsg"][gs, rr, :ln * B + ln].tobytes()
    for j in range(naggs):  # a dedicated aggregator holds the replies of exactly its slots
        z = res[m + j]
        for gs in range(j, G, A):
            for rr in range(int(rounds[gs])):
                assert int(z["rimm"][gs, rr]) == int(ref["rimm"][gs, rr]), (j, gs, rr)
