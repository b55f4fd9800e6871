"""The product's C++ multi-rank round (libomr_dist.so) with its ranks in SEPARATE PROCESSES sharing the one GPU,
over the HIP-IPC transport (omr_dist_create_ipc): device-side ordering between the ranks' streams (IPC events), no
stream synchronisation in the transport, in the synchronous, asynchronous (OMR_ROUND_ASYNC: the exchange on the
plan's second stream and second channel) and deferred (OMR_ROUND_DEFER) pipelines, every round a different input.
Each rank's outputs are checked bit for bit against the oracle: the rank-order block sums (server.cc:97-98), its
flags and next chain (client.cc:19-31) and the aggregator's union chain (server.cc:86-96)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from omr import Layout, cdist

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "ipc_round_worker.py")


def run_ranks(tmp_path, world, n, B, density, mode, pipe, rounds=3, workers=0, cycle=0, extra=()):
    uid = cdist.ipc_unique_id().hex()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.npz")
        outs.append(out)
        cmd = [sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--uid", uid, "--n", str(n),
               "--block", str(B), "--density", str(density), "--mode", str(mode), "--pipe", pipe,
               "--rounds", str(rounds), "--workers", str(workers), "--cycle", str(cycle), "--out", out] + list(extra)
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("an IPC rank hung:\n" + "\n".join(q.communicate()[0] or "" for q in procs))
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    assert not bad, "\n".join(f"rank {r} failed (rc {procs[r].returncode}):\n{logs[r][-2000:]}" for r in bad)
    return [np.load(o) for o in outs]


@pytest.mark.parametrize("world,pipe,mode,B,density,rounds", [
    (2, "sync", 0, 256, 0.095, 3),
    (3, "async", 0, 1024, 0.05, 3),
    (4, "defer", 0, 256, 0.3, 3),
    (4, "sync", 1, 512, 0.095, 3),
    (3, "defer", 1, 256, 0.5, 3),
    (2, "async", 2, 256, 0.2, 3),
    (4, "defer", 2, 256, 0.095, 3),
    # far more operations per channel than one ROCm IPC event survives (~32 records): the transport's event
    # generations, under the deferred pipeline, with the inputs and outputs reused every third round
    (3, "defer", 0, 256, 0.095, 60),
    (2, "async", 1, 256, 0.2, 45),
    # the progress thread (OMR_ROUND_THREAD) drives the transport
    (3, "thread", 0, 256, 0.095, 40),
    (4, "thread-async", 1, 512, 0.3, 9),
    (2, "thread", 2, 256, 0.2, 9),
])
def test_cpp_round_processes(gpu, tmp_path, world, pipe, mode, B, density, rounds):
    L = Layout(n=2 << 20, block_size=B)
    K = min(rounds, 3)
    res = run_ranks(tmp_path, world, L.n, B, density, mode, pipe, rounds, cycle=K)
    check_rounds(res, L, world, B, density, mode, rounds, K)


@pytest.mark.parametrize("world,pipe,mode", [(2, "sync", 0), (3, "defer", 1)])
def test_cpp_round_processes_replan(gpu, tmp_path, world, pipe, mode):
    """A plan destroyed and re-created on the same IPC transport: the new plan's buffers may reuse the old ones'
    addresses, so the transport must post them under new ids and its peers must map them afresh (a
    stale cached handle or mapping would move the old allocation's bytes without an error)."""
    L = Layout(n=2 << 20, block_size=256)
    res = run_ranks(tmp_path, world, L.n, 256, 0.2, mode, pipe, 3, cycle=3, extra=["--replan"])
    check_rounds(res, L, world, 256, 0.2, mode, 3, 3)


@pytest.mark.parametrize("world,pipe,mode", [(2, "defer", 0), (3, "sync", 1)])
def test_cpp_round_processes_replan_smaller(gpu, tmp_path, world, pipe, mode):
    """the second plan is SMALLER (2 MiB floats after 3 MiB: between 0.5 and 1 x), so the IPC transport hands
    it parked exported allocations up to twice its sizes (the lower_bound reuse), which keep their handles and ids; the
    peers must still address the right bytes of them.  Outputs bit-exact against the oracle."""
    L = Layout(n=2 << 20, block_size=256)
    res = run_ranks(tmp_path, world, L.n, 256, 0.2, mode, pipe, 3, cycle=3,
                    extra=["--replan", "--replan-first-n", str(3 << 20)])
    check_rounds(res, L, world, 256, 0.2, mode, 3, 3)


def check_rounds(res, L, world, B, density, mode, rounds, K):
    """Every rank's outputs of rounds 0..K-1 (inputs seeded rank + 10 round, as the worker makes them) against the
    oracle: rank-order block sums, flags, next chains and the union chain of the last round."""
    NB, P = L.num_lanes, L.num_threads
    bounds = [s * L.rows // world for s in range(world + 1)]
    for rd in range(K):
        bufs = [oracle.fill(oracle.gen_bitmap(w + 10 * rd, density, L.nb), B, mode=1, seed=w + 7 + 31 * rd)
                for w in range(world)]
        flags = [oracle.flags_from_data(b, B) for b in bufs]
        uf = oracle.union_flags(flags)
        for r in range(world):
            got = res[r][f"out{rd}"]
            if mode == 2:  # dense stand-in: every element of the rank's shard, rank-order sum
                exp = bufs[r].copy()
                lo, hi = bounds[r] * NB * B, bounds[r + 1] * NB * B
                acc = np.zeros(hi - lo, dtype=np.float32)
                for b in bufs:
                    acc = acc + b[lo:hi]
                exp[lo:hi] = acc
            else:
                full = bufs[r].copy()
                oracle.block_sum(bufs, L.n, B, NB, P, uf, full)
                if mode == 0:
                    exp = full
                else:  # reduce-scatter: the sums land in the rank's own shard only
                    exp = bufs[r].copy()
                    lo, hi = bounds[r] * NB * B, bounds[r + 1] * NB * B
                    exp[lo:hi] = full[lo:hi]
            assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"round {rd} rank {r} out"
            if rd == (rounds - 1) % K:  # the last round's flags and chains
                assert (res[r]["flags"] == flags[r]).all(), f"rank {r} flags"
                assert (res[r]["next"] == oracle.next_offsets(flags[r], L.n, B, NB, P)).all(), f"rank {r} next"
                assert (res[r]["unext"] == oracle.next_offsets(uf, L.n, B, NB, P)).all(), f"rank {r} union next"


@pytest.mark.parametrize("m,naggs,pipe,mode", [(2, 1, "sync", 0), (3, 2, "defer", 0), (2, 3, "async", 0),
                                               (3, 2, "sync", 1), (4, 1, "sync", 1)])
def test_dedicated_aggregators_processes(gpu, tmp_path, m, naggs, pipe, mode):
    """m worker processes + naggs dedicated aggregator processes (the reference's ./server machines, holding no
    tensor): all-reduce results on the workers; in reduce-scatter mode each aggregator's packed shard sums (write-set
    order: union blocks and lane heads of its rows, server.cc:143-147) and the workers' tensors left untouched."""
    B, density, rounds = 256, 0.2, 3
    L = Layout(n=2 << 20, block_size=B)
    world = m + naggs
    res = run_ranks(tmp_path, world, L.n, B, density, mode, pipe, rounds, workers=m)
    NB, P = L.num_lanes, L.num_threads
    bounds = [s * L.rows // naggs for s in range(naggs + 1)]
    heads = (np.arange(L.nb) // NB) % L.rows_per_part == 0
    for rd in range(rounds):
        bufs = [oracle.fill(oracle.gen_bitmap(w + 10 * rd, density, L.nb), B, mode=1, seed=w + 7 + 31 * rd)
                for w in range(m)]
        flags = [oracle.flags_from_data(b, B) for b in bufs]
        uf = oracle.union_flags(flags)
        full = np.zeros(L.n, dtype=np.float32)
        oracle.block_sum(bufs, L.n, B, NB, P, uf, full)
        for r in range(world):
            if r < m:
                got = res[r][f"out{rd}"]
                if mode == 0:
                    exp = bufs[r].copy()
                    oracle.block_sum(bufs, L.n, B, NB, P, uf, exp)
                else:
                    exp = bufs[r]
                assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"round {rd} worker {r}"
                if rd == rounds - 1:
                    assert (res[r]["next"] == oracle.next_offsets(flags[r], L.n, B, NB, P)).all()
            else:
                if rd == rounds - 1:
                    assert (res[r]["unext"] == oracle.next_offsets(uf, L.n, B, NB, P)).all(), f"aggregator {r}"
                if pipe == "sync":
                    j = r - m
                    sh, r0, r1 = res[r]["shard"]
                    assert (sh, r0, r1) == (j, bounds[j], bounds[j + 1])
                    blocks = np.arange(r0 * NB, r1 * NB)
                    sel = blocks[(uf.astype(bool) | heads)[r0 * NB:r1 * NB]]
                    exp = full.reshape(L.nb, B)[sel].reshape(-1)
                    assert (res[r][f"sums{rd}"].view(np.uint32) == exp.view(np.uint32)).all(), f"agg {j} round {rd}"
