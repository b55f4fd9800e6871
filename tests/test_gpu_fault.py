"""Failure containment: a rank that fails, or whose peer is stuck or gone, returns an
error within the transport's deadline instead of blocking, and its peers are not left waiting on it.  The reference
exits on a failed post (common.cc:450-451); here a failed transport is ABORTED (include/omr_dist.h):

* RCCL, one-rank communicator in this process: a failed exchange closes its group (a group left open would capture a
  later communicator's calls), aborts both communicators (ncclCommAbort), and every later call fails at once with
  OMR_EABORTED; a new communicator then runs a round bit-exact against the oracle.  omr_ar_plan_wait past the
  deadline aborts too (world 1: the RCCL abort path with nothing queued on the communicators).
* Loopback, two ranks as threads: a one-sided fault before (or after) the faulting rank's first piece ends the HEALTHY
  rank's round with an error at once (the group's abort flag), in synchronous and deferred rounds; a silent peer ends
  it at the deadline; a round failing in its first half leaves later threaded, deferred rounds failing
  fast instead of hanging; a fresh group afterwards is bit-exact.
* HIP IPC, two processes: the same one-sided fault, across processes (tests/ipc_round_worker.py --fault-*)."""
import ctypes
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, cdist
from omr._lib import OmrError

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
EABORTED, ETIMEDOUT = -2, -3


def _round_matches_oracle(eng, gpu, L, seed=5):
    x = oracle.fill(oracle.gen_bitmap(0, 0.2, L.nb), 256, mode=1, seed=seed)
    xd = torch.from_numpy(x).to(gpu)
    out = xd.clone()
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    eng.run(xd, out=out, next_offsets=nxt, mode=1)
    torch.cuda.synchronize()
    f = oracle.flags_from_data(x, 256)
    exp = x.copy()
    oracle.block_sum([x], L.n, 256, L.num_lanes, 8, f, exp)
    assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all()
    assert (nxt.cpu().numpy().view(np.uint32) == oracle.next_offsets(f, L.n, 256, L.num_lanes, 8)).all()


@pytest.mark.parametrize("rccl_calls", [False, True])
def test_rccl_failed_exchange_aborts(gpu, rccl_calls):
    """rccl_calls: the one-rank communicator issues its collectives as RCCL calls (omr_dist_test_world1_round), so the
    failed exchange is inside ncclGroupStart / ncclGroupEnd and the abort runs ncclCommAbort after RCCL calls were made
    on both communicators (world 1's copies bypass RCCL otherwise)."""
    L = Layout(n=1 << 20, block_size=256)
    eng = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        if rccl_calls:
            eng.test_world1_round(True)
            src = torch.arange(64, dtype=torch.int32, device=gpu)
            dst = torch.zeros(64, dtype=torch.int32, device=gpu)
            eng.allgather(src, dst)  # an RCCL all-gather on `comm`
            assert eng.exchange([None], [None]) == 0  # an empty RCCL group on `xcomm`
            torch.cuda.synchronize()
            assert torch.equal(src, dst)
        _round_matches_oracle(eng, gpu, L)
        eng.inject_fault(0)
        t0 = time.monotonic()
        assert eng.exchange([None], [None]) != 0  # failed inside the RCCL group: the group is closed, then aborted
        assert eng.aborted
        src = torch.arange(64, dtype=torch.int32, device=gpu)
        dst = torch.zeros(64, dtype=torch.int32, device=gpu)
        with pytest.raises(OmrError, match="aborted"):
            eng.allgather(src, dst)
        with pytest.raises(OmrError, match="aborted"):
            eng.run(src.float().repeat(L.n // 64), mode=1)
        assert time.monotonic() - t0 < 10
    finally:
        eng.close()  # destroying an aborted transport does not wait on anything
    # a group left open by the failed exchange would capture this communicator's all-gather (never launched)
    eng2 = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        if rccl_calls:
            eng2.test_world1_round(True)
        src = torch.arange(64, dtype=torch.int32, device=gpu)
        dst = torch.zeros(64, dtype=torch.int32, device=gpu)
        eng2.allgather(src, dst)
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
        _round_matches_oracle(eng2, gpu, L, seed=6)
    finally:
        eng2.close()


def _sleep_cycles_for(seconds):
    """torch.cuda._sleep cycles that keep the stream busy for about `seconds` (calibrated here: the GPU's clock)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cyc = 20_000_000
    a.record()
    torch.cuda._sleep(cyc)
    b.record()
    torch.cuda.synchronize()
    per_s = cyc / (a.elapsed_time(b) * 1e-3)
    return int(per_s * seconds)


@pytest.mark.parametrize("layout", ["one side stream", "N>1 streams"])
def test_rccl_world1_calls_round(gpu, layout):
    """With RCCL calls kept at world 1 (omr_dist_test_world1_round), the rounds that use the transport at world 1 -- the
    dense stand-in (ncclReduceScatter) and a bucket round (ncclAllGather of the masks, an empty grouped exchange) --
    are bit-exact against the oracle; on the plan made before the hook (one side stream) and on one made after it (the
    N > 1 layout: the exchange stream waits for the plan stream)."""
    B = 256
    L = Layout(n=1 << 20, block_size=B)
    eng = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        eng.test_world1_round(True)
        if layout == "N>1 streams":
            eng.replan()
        x = oracle.fill(oracle.gen_bitmap(0, 0.3, L.nb), B, mode=1, seed=4)
        f = oracle.flags_from_data(x, B)
        exp = x.copy()
        oracle.block_sum([x], L.n, B, L.num_lanes, 8, f, exp)
        xd = torch.from_numpy(x).to(gpu)
        for mode in (0, 1):  # the multi-rank round's path at world 1: all-gather, plan, empty exchange, shard sum
            out = xd.clone()
            eng.run(xd, out=out, mode=mode, async_=True, defer=True)
            eng.join()
            torch.cuda.synchronize()
            assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all(), mode
        out = torch.zeros_like(xd)
        eng.run(xd, out=out, mode=2)  # dense reduce-scatter over one rank: the tensor itself
        torch.cuda.synchronize()
        assert (out.cpu().numpy().view(np.uint32) == x.view(np.uint32)).all()
        buf = torch.from_numpy(np.concatenate([x, x])).to(gpu)
        eng.run_buckets(buf, mode=0)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        for k in range(2):
            assert (got[k * L.n:(k + 1) * L.n].view(np.uint32) == exp.view(np.uint32)).all(), k
    finally:
        eng.close()


@pytest.mark.parametrize("transport", ["rccl1", "local1"])
def test_abort_from_another_thread_during_wait(gpu, transport):
    """omr_dist_abort from a second thread while the owner waits in omr_ar_plan_wait (the abort must not
    free an RCCL communicator that the waiting thread's poll is using): the wait ends with an error well before its
    deadline, the transport is aborted, and closing it returns."""
    L = Layout(n=1 << 20, block_size=256)
    eng = cdist.CppSparseAllreduce(L, gpu, transport=transport)
    try:
        _round_matches_oracle(eng, gpu, L)
        eng.set_timeout(20000)
        torch.cuda._sleep(_sleep_cycles_for(2.0))
        t = threading.Thread(target=lambda: (time.sleep(0.3), eng.abort()), daemon=True)
        t0 = time.monotonic()
        t.start()
        with pytest.raises(OmrError, match="abort"):
            eng.wait()
        t.join(timeout=30)
        assert not t.is_alive()
        assert eng.aborted
        assert time.monotonic() - t0 < 10.0
        torch.cuda.synchronize()  # the sleep ends by itself
    finally:
        eng.close()


@pytest.mark.parametrize("transport", ["rccl1", "local1"])
def test_wait_past_deadline_aborts(gpu, transport):
    """omr_ar_plan_wait on a stream that does not drain within the deadline returns OMR_ETIMEDOUT and aborts the
    transport (nothing is queued on the communicators: the stream is held by a bounded GPU sleep)."""
    L = Layout(n=1 << 20, block_size=256)
    eng = cdist.CppSparseAllreduce(L, gpu, transport=transport)
    try:
        _round_matches_oracle(eng, gpu, L)
        cycles = _sleep_cycles_for(2.5)
        eng.set_timeout(400)
        torch.cuda._sleep(cycles)
        t0 = time.monotonic()
        with pytest.raises(OmrError, match=f"rc={ETIMEDOUT}"):
            eng.wait()
        # the wait ends at its deadline; ncclCommAbort then synchronises the device, i.e. waits for the sleep to end
        # (a hung RCCL kernel would instead see the abort flag and leave): about the sleep's length for rccl1
        assert time.monotonic() - t0 < (5.0 if transport == "rccl1" else 2.0)
        assert eng.aborted and eng.failed == ETIMEDOUT
        with pytest.raises(OmrError, match="failed in an earlier round|aborted"):
            eng.run(torch.zeros(L.n, device=gpu), mode=1)
        torch.cuda.synchronize()  # the sleep ends by itself
    finally:
        eng.close()


def _loopback_group(D, world, L, timeout_ms):
    board = D.omr_local_board_create(world)
    ds, plans = [], []
    for r in range(world):
        d, p = ctypes.c_void_p(), ctypes.c_void_p()
        assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
        assert D.omr_dist_set_timeout(d, timeout_ms) == 0
        assert D.omr_ar_plan_create(d, L.n, 256, L.num_lanes, 8, ctypes.byref(p)) == 0
        ds.append(d)
        plans.append(p)
    return board, ds, plans


def _run_threads(fn, world, limit):
    errs, th = [], []

    def wrap(r):
        try:
            fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append(f"rank {r}: {e!r}")
    th = [threading.Thread(target=wrap, args=(r,), daemon=True) for r in range(world)]
    t0 = time.monotonic()
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=max(1.0, limit - (time.monotonic() - t0)))
    assert not any(t.is_alive() for t in th), f"a rank was still blocked after {limit} s"
    assert not errs, errs
    return time.monotonic() - t0


def _check_fresh_group(D, gpu, bufs, L, mode):
    """A new group after the failure: one round per rank, bit-exact against the oracle."""
    world, B = len(bufs), 256
    board, ds, plans = _loopback_group(D, world, L, 60000)
    outs = [None] * world

    def rank(r):
        torch.cuda.set_device(0)
        x = torch.from_numpy(bufs[r].copy()).cuda()
        out = x.clone()
        st = torch.cuda.Stream()
        rc = D.omr_sparse_round_f32(plans[r], x.data_ptr(), out.data_ptr(), None, None, None, mode, None, None,
                                    st.cuda_stream)
        assert rc == 0, D.omr_dist_last_error()
        st.synchronize()
        outs[r] = out.cpu().numpy()
    _run_threads(rank, world, 120)
    for r in range(world):
        D.omr_ar_plan_destroy(plans[r])
        D.omr_dist_destroy(ds[r])
    D.omr_local_board_destroy(board)
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    bounds = [s * L.rows // world for s in range(world + 1)]
    rowf = L.num_lanes * B
    for r in range(world):
        full = bufs[r].copy()
        oracle.block_sum(bufs, L.n, B, L.num_lanes, 8, uf, full)
        exp = bufs[r].copy()
        if mode == 1:
            exp[bounds[r] * rowf:bounds[r + 1] * rowf] = full[bounds[r] * rowf:bounds[r + 1] * rowf]
        else:
            exp = full
        assert (outs[r].view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r}"


@pytest.mark.parametrize("after,mode", [
    (0, 0),        # the faulting rank stops before its first piece, all-reduce
    (1, 1),        # ... after its only piece (the peer already copied it), reduce-scatter
    (0, 0x401),    # deferred reduce-scatter rounds: the failing exchange is issued by a later call
])
def test_loopback_one_sided_fault(gpu, after, mode):
    world, L = 2, Layout(n=2 << 20, block_size=256)
    D = cdist.load()
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), 256, mode=1, seed=w + 11) for w in range(world)]
    board, ds, plans = _loopback_group(D, world, L, 20000)
    rcs = [[] for _ in range(world)]
    assert D.omr_dist_inject_fault(ds[1], after) == 0

    def rank(r):
        torch.cuda.set_device(0)
        x = torch.from_numpy(bufs[r].copy()).cuda()
        st = torch.cuda.Stream()
        res = [x.clone() for _ in range(3)]
        for k in range(3 if mode & 0x400 else 1):
            rcs[r].append(D.omr_sparse_round_f32(plans[r], x.data_ptr(), res[k].data_ptr(), None, None, None, mode,
                                                 None, None, st.cuda_stream))
        rcs[r].append(D.omr_ar_plan_wait(plans[r], st.cuda_stream))
    took = _run_threads(rank, world, 60)
    assert took < 15, f"the healthy rank took {took:.1f} s (the group's abort flag should end its wait at once)"
    for r in range(world):
        assert any(rc != 0 for rc in rcs[r]), (r, rcs[r])  # the healthy rank 0 too: it got an error, not a hang
        assert D.omr_ar_plan_failed(plans[r]) != 0
        assert D.omr_dist_aborted(ds[r]) == 1
        D.omr_ar_plan_destroy(plans[r])
        D.omr_dist_destroy(ds[r])
    D.omr_local_board_destroy(board)
    _check_fresh_group(D, gpu, bufs, L, mode & 0xFF)


def test_loopback_silent_peer_deadline(gpu):
    """Rank 1 does not show up for 4 s: rank 0's round ends at its 1 s deadline with OMR_ETIMEDOUT (and aborts the
    group), and rank 1's late round fails at once."""
    world, L = 2, Layout(n=1 << 20, block_size=256)
    D = cdist.load()
    board, ds, plans = _loopback_group(D, world, L, 1000)
    rcs, took = [None] * world, [None] * world

    def rank(r):
        torch.cuda.set_device(0)
        x = torch.zeros(L.n, device="cuda")
        st = torch.cuda.Stream()
        if r == 1:
            time.sleep(4)
        t0 = time.monotonic()
        rcs[r] = D.omr_sparse_round_f32(plans[r], x.data_ptr(), x.data_ptr(), None, None, None, 0, None, None,
                                        st.cuda_stream)
        took[r] = time.monotonic() - t0
    _run_threads(rank, world, 60)
    assert rcs[0] == ETIMEDOUT and took[0] < 3.0, (rcs, took)
    assert rcs[1] == EABORTED and took[1] < 1.0, (rcs, took)
    for r in range(world):
        D.omr_ar_plan_destroy(plans[r])
        D.omr_dist_destroy(ds[r])
    D.omr_local_board_destroy(board)


def test_loopback_first_half_failure_then_threaded_rounds(gpu):
    """a non-threaded round failing in its first half (its all-gather), followed by threaded deferred
    rounds (the fused pack's wait for the second halves): every later call returns an error promptly, join and
    destroy return, nothing hangs."""
    world, L = 2, Layout(n=2 << 20, block_size=256)
    D = cdist.load()
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), 256, mode=1, seed=w + 3) for w in range(world)]
    board, ds, plans = _loopback_group(D, world, L, 20000)
    assert D.omr_ar_plan_fused_pack(plans[0]) == 1
    assert D.omr_dist_inject_allgather_fault(ds[0]) == 0
    rcs = [[] for _ in range(world)]

    def rank(r):
        torch.cuda.set_device(0)
        x = torch.from_numpy(bufs[r].copy()).cuda()
        st = torch.cuda.Stream()
        out = x.clone()
        rcs[r].append(D.omr_sparse_round_f32(plans[r], x.data_ptr(), out.data_ptr(), None, None, None, 0, None, None,
                                             st.cuda_stream))
        for _ in range(4):  # OMR_ROUND_THREAD | OMR_ROUND_DEFER | OMR_ROUND_TIME_EXCHANGE, reduce-scatter
            rcs[r].append(D.omr_sparse_round_f32(plans[r], x.data_ptr(), out.data_ptr(), None, None, None,
                                                 0x800 | 0x400 | 0x200 | 1, None, None, st.cuda_stream))
        rcs[r].append(D.omr_ar_plan_join(plans[r], st.cuda_stream))
        ms = (ctypes.c_float * 4)()
        D.omr_ar_plan_stage_timings(plans[r], ms, None, None, None)  # returns (no open record blocks it)
        st.synchronize()
    took = _run_threads(rank, world, 60)
    assert took < 15
    for r in range(world):
        assert rcs[r][0] != 0 and all(rc != 0 for rc in rcs[r][1:]), (r, rcs[r])
        D.omr_ar_plan_destroy(plans[r])
        D.omr_dist_destroy(ds[r])
    D.omr_local_board_destroy(board)
    _check_fresh_group(D, gpu, bufs, L, 0)


WORKER = os.path.join(HERE, "ipc_round_worker.py")


@pytest.mark.parametrize("after,pipe", [(0, "sync"), (0, "defer")])
def test_ipc_one_sided_fault(gpu, tmp_path, after, pipe):
    """Two processes over HIP IPC; rank 1's exchange fails before its first piece.  Rank 0 must get an error well
    within the deadline (rank 1's abort flag on the board), and both processes must exit."""
    world, n = 2, 2 << 20
    uid = cdist.ipc_unique_id().hex()
    procs = []
    for r in range(world):
        cmd = [sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--uid", uid, "--n", str(n),
               "--density", "0.2", "--mode", "0", "--pipe", pipe, "--rounds", "3", "--timeout-ms", "30000",
               "--fault-rank", "1", "--fault-after", str(after), "--status", str(tmp_path / f"s{r}.json"),
               "--out", str(tmp_path / f"r{r}.npz")]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=200)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("an IPC rank hung after the one-sided fault")
    st = [json.load(open(tmp_path / f"s{r}.json")) for r in range(world)]
    assert "fault injected" in st[1]["error"], (st, logs)
    assert st[0]["error"], f"the healthy rank reported no error: {st} {logs}"
    assert st[0]["seconds_to_error"] < 20, st
    for r, p in enumerate(procs):
        assert p.returncode == 3, f"rank {r} exit {p.returncode}:\n{logs[r]}"


def test_ipc_destroy_bounded_while_peer_silent(gpu, tmp_path):
    """Two processes over HIP IPC; rank 1's stream is held by a 12 s kernel queued before its first round, so rank 0's
    stream waits on the device for rank 1's part of the all-gather while both hosts run on.  With a 2 s deadline rank 0
    fails (no counts), aborts, and closes: plan and transport teardown must end within their deadlines (reporting
    OMR_ETIMEDOUT and leaving the device memory allocated) instead of waiting for the device.  Both ranks
    then drain the device (the kernel ends and every wait resolves) before they leave."""
    world, n = 2, 2 << 20
    uid = cdist.ipc_unique_id().hex()
    procs = []
    for r in range(world):
        cmd = [sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--uid", uid, "--n", str(n),
               "--density", "0.2", "--mode", "0", "--pipe", "sync", "--rounds", "2", "--timeout-ms", "2000",
               "--stall-ms", "12000" if r == 1 else "0", "--drain", "--status", str(tmp_path / f"s{r}.json"),
               "--out", str(tmp_path / f"r{r}.npz")]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=200)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("an IPC rank hung")
    st = [json.load(open(tmp_path / f"s{r}.json")) for r in range(world)]
    for r, p in enumerate(procs):
        assert p.returncode == 3, f"rank {r} exit {p.returncode}:\n{logs[r]}"
    assert st[0]["error"] and st[0]["seconds_to_error"] < 6, (st, logs)
    # two bounded waits of 2 s (plan, transport), well short of the 12 s the device stays busy
    assert st[0]["close_seconds"] < 7, (st, logs)
    assert st[0]["close_rcs"] == [ETIMEDOUT, ETIMEDOUT], (st, logs)
