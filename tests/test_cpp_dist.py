"""C++ host path (libomr_dist.so, ./omr_client, ./omr_server) on the GPU.

The multi-rank round in C++ is checked against the oracle with the in-process loopback transport (several ranks
as threads sharing one GPU), and the two CLI drivers are run end to end: loopback workers with the working
CHECK (-c), and a server + one RCCL worker over the TCP rendezvous.  (RCCL refuses two ranks on one GPU, so the
multi-rank RCCL leg runs on multi-GPU nodes only.)"""
import ctypes
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, _lib

pytestmark = pytest.mark.gpu
PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "omnireduce-rdma-demo_amd")
BIN = os.path.join(PKG, "bin")


def dist_lib():
    _lib.load()
    L = ctypes.CDLL(os.path.join(PKG, "omr", "libomr_dist.so"))
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.omr_local_board_create.restype = vp
    L.omr_local_board_create.argtypes = [i]
    L.omr_local_board_destroy.argtypes = [vp]
    L.omr_dist_create_local.argtypes = [vp, i, vp]
    L.omr_dist_destroy.argtypes = [vp]
    L.omr_ar_plan_create.argtypes = [vp, u64, u32, u32, u32, vp]
    L.omr_ar_plan_destroy.argtypes = [vp]
    L.omr_sparse_allreduce_f32.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.omr_sparse_round_f32.argtypes = [vp, vp, vp, vp, vp, vp, i, vp, vp, vp]
    L.omr_ar_plan_join.argtypes = [vp, vp]
    L.omr_ar_plan_exchange_time.argtypes = [vp, vp, vp, vp]
    L.omr_ar_plan_device_bytes.restype = u64
    L.omr_ar_plan_device_bytes.argtypes = [vp]
    L.omr_ar_plan_set_side_streams.argtypes = [vp, i]
    L.omr_ar_plan_side_streams.argtypes = [vp]
    L.omr_dist_last_error.restype = ctypes.c_char_p
    return L


@pytest.mark.parametrize("world,B,density", [(2, 256, 0.095), (3, 1024, 0.0099), (4, 512, 0.49),
                                                   (8, 256, 0.095),
                                                   # world sizes that do not divide the 128 rows (ragged shards), and
                                                   # the largest group the shard sum takes (OMR_MAX_WORKERS)
                                                   (5, 256, 0.3), (6, 512, 0.095), (7, 256, 0.2), (16, 256, 0.095)])
def test_cpp_round_loopback(gpu, world, B, density):
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B, mode=1, seed=w + 7) for w in range(world)]
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    board = D.omr_local_board_create(world)
    errs, results = [], [None] * world

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = torch.from_numpy(bufs[r].copy()).cuda()
            out = x.clone()
            flags = torch.empty(L.nb, dtype=torch.int32, device="cuda")
            nxt = torch.empty(L.nb, dtype=torch.int32, device="cuda")
            unext = torch.empty(L.nb, dtype=torch.int32, device="cuda")
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            for _ in range(2):
                rc = D.omr_sparse_allreduce_f32(plan, x.data_ptr(), out.data_ptr(), flags.data_ptr(), nxt.data_ptr(),
                                                unext.data_ptr(), None, None, st.cuda_stream)
                assert rc == 0, D.omr_dist_last_error()
            torch.cuda.synchronize()
            results[r] = (out.cpu().numpy(), flags.cpu().numpy(), nxt.cpu().numpy().view(np.uint32),
                          unext.cpu().numpy().view(np.uint32))
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    un = oracle.next_offsets(uf, L.n, B, L.num_lanes, 8)
    for r in range(world):
        exp = bufs[r].copy()
        oracle.block_sum(bufs, L.n, B, L.num_lanes, 8, uf, exp)
        out, fl, nx, unx = results[r]
        assert (out.view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r} sum"
        f = oracle.flags_from_data(bufs[r], B)
        assert (fl == f).all()
        assert (nx == oracle.next_offsets(f, L.n, B, L.num_lanes, 8)).all()
        assert (unx == un).all()


@pytest.mark.parametrize("B,density", [(256, 0.095), (1024, 1.0)])
def test_cpp_round_world1_counts_optional(gpu, B, density):
    """A one-rank round asked for no counts does not wait for them (its one launch is the round): rounds with and
    without count pointers interleaved on one plan, each bit-exact against the oracle, and every round that asks gets
    the write-set size (the worker's non-zero blocks and every partition's lane heads) while the publications of the
    rounds that did not ask are carried by the next scan."""
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    buf = oracle.fill(oracle.gen_bitmap(0, density, L.nb), B, mode=1, seed=3)
    f = oracle.flags_from_data(buf, B)
    exp = buf.copy()
    oracle.block_sum([buf], L.n, B, L.num_lanes, 8, f, exp)
    rows = L.nb // L.num_lanes
    head = ((np.arange(L.nb) // L.num_lanes) % (rows // 8)) == 0
    ws = int(np.count_nonzero((f != 0) | head))
    board = D.omr_local_board_create(1)
    d, plan = ctypes.c_void_p(), ctypes.c_void_p()
    assert D.omr_dist_create_local(board, 0, ctypes.byref(d)) == 0
    assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
    try:
        x = torch.from_numpy(buf.copy()).cuda()
        outs = [torch.full_like(x, float("nan")) for _ in range(3)]
        st = torch.cuda.Stream()
        sent, uni = ctypes.c_uint64(7), ctypes.c_uint64(7)
        for k, want in enumerate([False, False, True, False, True, True, False]):
            out = outs[k % 3]
            out.copy_(x)
            torch.cuda.synchronize()
            uni.value = 7
            rc = D.omr_sparse_allreduce_f32(plan, x.data_ptr(), out.data_ptr(), None, None, None,
                                            ctypes.byref(sent) if want else None, ctypes.byref(uni) if want else None,
                                            st.cuda_stream)
            assert rc == 0, D.omr_dist_last_error()
            st.synchronize()
            assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all(), f"round {k}"
            if want:
                assert (sent.value, uni.value) == (0, ws), f"round {k}"
    finally:
        D.omr_ar_plan_destroy(plan)
        D.omr_dist_destroy(d)
        D.omr_local_board_destroy(board)


@pytest.mark.parametrize("world,mode", [(3, 0), (4, 1), (5, 0)])
def test_cpp_round_side_streams_switch(gpu, world, mode):
    """Pipelined rounds (async | defer) with the side streams switched between them (omr_ar_plan_set_side_streams:
    2 -> 1 -> 2, and ragged shards at world 3 and 5, where a pack pass on the plan stream reuses send buffers the
    exchange stream read): every round's output bit-exact against the oracle, inputs different per round."""
    B = 256
    L = Layout(n=1 << 20, block_size=B)
    D = dist_lib()
    K = 4  # rounds per layout phase, each on its own input
    phases = [2, 1, 2]
    nr = K * len(phases)
    bufs = [[oracle.fill(oracle.gen_bitmap(w + 10 * k, 0.3, L.nb), B, mode=1, seed=w + 31 * k) for w in range(world)]
            for k in range(nr)]
    board = D.omr_local_board_create(world)
    errs, outs = [], [None] * world

    def rank(r):
        try:
            torch.cuda.set_device(0)
            xs = [torch.from_numpy(bufs[k][r].copy()).cuda() for k in range(nr)]
            os_ = [x.clone() for x in xs]
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            assert D.omr_ar_plan_side_streams(plan) == 2  # the default at world > 1
            st = torch.cuda.Stream()
            k = 0
            for n in phases:
                assert D.omr_ar_plan_set_side_streams(plan, n) == 0, D.omr_dist_last_error()
                assert D.omr_ar_plan_side_streams(plan) == n
                for _ in range(K):
                    rc = D.omr_sparse_round_f32(plan, xs[k].data_ptr(), os_[k].data_ptr(), None, None, None,
                                                mode | 0x100 | 0x400, None, None, st.cuda_stream)
                    assert rc == 0, D.omr_dist_last_error()
                    k += 1
            assert D.omr_ar_plan_set_side_streams(plan, 3) != 0
            assert D.omr_ar_plan_join(plan, st.cuda_stream) == 0
            torch.cuda.synchronize()
            outs[r] = [o.cpu().numpy() for o in os_]
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    bounds = [s * L.rows // world for s in range(world + 1)]
    rowf = L.num_lanes * B
    for k in range(nr):
        uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs[k]])
        for r in range(world):
            full = bufs[k][r].copy()
            oracle.block_sum(bufs[k], L.n, B, L.num_lanes, 8, uf, full)
            if mode == 0:
                exp = full
            else:
                exp = bufs[k][r].copy()
                lo, hi = bounds[r] * rowf, bounds[r + 1] * rowf
                exp[lo:hi] = full[lo:hi]
            assert (outs[r][k].view(np.uint32) == exp.view(np.uint32)).all(), f"round {k} rank {r}"


@pytest.mark.parametrize("world,rounds", [(3, 1), (8, 3)])
def test_cpp_reduce_scatter_loopback(gpu, world, rounds):
    """Reduce-scatter mode (the bench's N>1 step); world 8 = the driver's 8-GPU scale run as threads on one GPU,
    several rounds back to back (the plan's per-round state must reset)."""
    B = 256
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), B, mode=1, seed=w + 3) for w in range(world)]
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    board = D.omr_local_board_create(world)
    errs, outs = [], [None] * world

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = torch.from_numpy(bufs[r].copy()).cuda()
            out = x.clone()
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            for _ in range(rounds):  # x is never written: every round writes the same shard sums into out
                assert D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), None, None, None, 1, None, None,
                                              st.cuda_stream) == 0, D.omr_dist_last_error()
            torch.cuda.synchronize()
            outs[r] = out.cpu().numpy()
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    bounds = [s * L.rows // world for s in range(world + 1)]
    for r in range(world):
        full = bufs[r].copy()
        oracle.block_sum(bufs, L.n, B, L.num_lanes, 8, uf, full)
        exp = bufs[r].copy()
        lo, hi = bounds[r] * L.num_lanes * B, bounds[r + 1] * L.num_lanes * B
        exp[lo:hi] = full[lo:hi]
        assert (outs[r].view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r}"


A, D_, T = 0x100, 0x400, 0x800  # OMR_ROUND_ASYNC, OMR_ROUND_DEFER, OMR_ROUND_THREAD


@pytest.mark.parametrize("world,mode,round_flags", [
    (3, 1, (A,) * 7), (8, 1, (A,) * 7), (4, 0, (A,) * 7), (3, 1, (A, A, 0, A, 0)),
    (3, 1, (D_,) * 7), (8, 1, (D_,) * 7), (4, 0, (D_,) * 7), (4, 2, (D_,) * 7),
    (3, 1, (D_, D_, 0, D_, A)), (4, 0, (A, D_, D_, A, D_, D_, D_)), (3, 0, (D_, D_, D_, 0, D_, D_, A, D_)),
    # the progress thread (OMR_ROUND_THREAD), alone and mixed with calls that must first drain it
    (3, 1, (T,) * 7), (8, 1, (T | D_,) * 7), (4, 2, (T | D_,) * 7),
    (4, 0, (T | D_, T | D_, 0, T, D_, T | D_, A, T | D_)), (3, 1, (T | D_, A, T, T | D_, T | D_, 0, T))])
def test_cpp_async_rounds_loopback(gpu, world, mode, round_flags):
    """OMR_ROUND_ASYNC: the bookkeeping of round k runs on the plan stream and its exchange and sums on the
    communication stream while round k+1 scans; rounds take different inputs and outputs (the bench's rotation),
    use the three plan buffer sets in turn (seven rounds: every set refilled), and are joined once at the end.
    OMR_ROUND_DEFER: round k's exchange is issued by call k+2 (or a call without the flag, or the join).  Rounds
    issued without a flag in between must first finish the deferred rounds and wait for the asynchronous ones
    before using the stream.  OMR_ROUND_THREAD: the plan's progress thread issues everything after each scan; a
    call without it first waits until the thread has issued every queued round."""
    B, rounds = 256, len(round_flags)
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    bufs = [[oracle.fill(oracle.gen_bitmap(w + 10 * k, 0.15, L.nb), B, mode=1, seed=w + 10 * k + 1)
             for w in range(world)] for k in range(rounds)]
    board = D.omr_local_board_create(world)
    errs, outs = [], [[None] * rounds for _ in range(world)]

    def rank(r):
        try:
            torch.cuda.set_device(0)
            xs = [torch.from_numpy(bufs[k][r].copy()).cuda() for k in range(rounds)]
            os_ = [x.clone() for x in xs]
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            for k in range(rounds):
                flag = round_flags[k]
                assert D.omr_sparse_round_f32(plan, xs[k].data_ptr(), os_[k].data_ptr(), None, None, None,
                                              mode | flag, None, None, st.cuda_stream) == 0, D.omr_dist_last_error()
            assert D.omr_ar_plan_join(plan, st.cuda_stream) == 0
            st.synchronize()
            for k in range(rounds):
                outs[r][k] = os_[k].cpu().numpy()
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    bounds = [s * L.rows // world for s in range(world + 1)]
    for k in range(rounds):
        uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs[k]])
        for r in range(world):
            full = bufs[k][r].copy()
            oracle.block_sum(bufs[k], L.n, B, L.num_lanes, 8, uf, full)
            if mode in (1, 2):  # reduce-scatter, sparse or dense: this shard's sums, other rows untouched
                exp = bufs[k][r].copy()
                lo, hi = bounds[r] * L.num_lanes * B, bounds[r + 1] * L.num_lanes * B
                exp[lo:hi] = full[lo:hi]
            else:
                exp = full
            assert (outs[r][k].view(np.uint32) == exp.view(np.uint32)).all(), f"round {k} rank {r}"


@pytest.mark.parametrize("world,flags", [(4, 0), (8, 0x100)])
def test_cpp_dense_reduce_scatter_loopback(gpu, world, flags):
    """OMR_ROUND_DENSE_REDUCE_SCATTER (the dense stand-in): this rank's shard of the elementwise rank-order sum of
    every worker's whole tensor; other rows untouched; the worker outputs as in the sparse modes."""
    B = 256
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.3, L.nb), B, mode=1, seed=w + 5) for w in range(world)]
    dense = np.zeros(L.n, dtype=np.float32)
    for b in bufs:
        dense = dense + b
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    board = D.omr_local_board_create(world)
    errs, outs = [], [None] * world

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = torch.from_numpy(bufs[r].copy()).cuda()
            out = x.clone()
            unext = torch.empty(L.nb, dtype=torch.int32, device="cuda")
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            for _ in range(2):
                assert D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), None, None, unext.data_ptr(),
                                              2 | flags, None, None, st.cuda_stream) == 0, D.omr_dist_last_error()
            assert D.omr_ar_plan_join(plan, st.cuda_stream) == 0
            st.synchronize()
            outs[r] = (out.cpu().numpy(), unext.cpu().numpy().view(np.uint32))
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    un = oracle.next_offsets(uf, L.n, B, L.num_lanes, 8)
    bounds = [s * L.rows // world for s in range(world + 1)]
    for r in range(world):
        exp = bufs[r].copy()
        lo, hi = bounds[r] * L.num_lanes * B, bounds[r + 1] * L.num_lanes * B
        exp[lo:hi] = dense[lo:hi]
        out, unx = outs[r]
        assert (out.view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r}"
        assert (unx == un).all()


def test_cpp_dense_reduce_scatter_needs_equal_shards(gpu):
    D = dist_lib()
    board = D.omr_local_board_create(3)
    d, plan = ctypes.c_void_p(), ctypes.c_void_p()
    assert D.omr_dist_create_local(board, 0, ctypes.byref(d)) == 0
    L = Layout(n=2 << 20, block_size=256)  # 128 rows: not a multiple of 3
    assert D.omr_ar_plan_create(d, L.n, 256, L.num_lanes, 8, ctypes.byref(plan)) == 0
    x = torch.zeros(L.n, device="cuda")
    rc = D.omr_sparse_round_f32(plan, x.data_ptr(), x.data_ptr(), None, None, None, 2, None, None, None)
    assert rc != 0 and b"equal shards" in D.omr_dist_last_error()
    D.omr_ar_plan_destroy(plan)
    D.omr_dist_destroy(d)
    D.omr_local_board_destroy(board)


def _run(cmd, timeout=300):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_client_loopback_cli(gpu):
    rc, out = _run([os.path.join(BIN, "omr_client"), "-L", "3", "-n", str(4 << 20), "-r", "0.095", "-W", "2",
                    "-R", "4", "-c"])
    assert rc == 0, out
    assert "check OK" in out and "average alg bw" in out and "test result is 0" in out


@pytest.mark.parametrize("mode", [[], ["-M"]])
def test_client_loopback_check_in_place(gpu, mode):
    """-c with -I: the in-place rounds would compound (0.01 -> 0.03 -> 0.09 at three workers), so each round starts
    from the generator's input again, as the reference's CHECK restores res.buf = input (client.cc:463-464)."""
    rc, out = _run([os.path.join(BIN, "omr_client"), "-L", "3", "-n", str(1 << 20), "-r", "0.3", "-W", "2",
                    "-R", "3", "-c", "-I"] + mode)
    assert rc == 0, out
    assert "check OK" in out and "test result is 0" in out


@pytest.mark.parametrize("workers,r", [(1, "0.095"), (1, "1.0"), (3, "0.3")])
def test_client_loopback_host_resident(gpu, workers, r):
    """-H: each worker's tensor lives in pinned host memory, as the reference's registered res->buf, and every round
    reads it and returns its results into it (one worker: one launch per round on the mapped buffer; three: staged
    through device buffers); the CHECK restores the input before each round and checks the last one."""
    rc, out = _run([os.path.join(BIN, "omr_client"), "-L", str(workers), "-H", "-n", str(1 << 20), "-r", r, "-W", "2",
                    "-R", "3", "-c"])
    assert rc == 0, out
    assert "check OK" in out and "average alg bw" in out and "test result is 0" in out


def test_client_host_with_messages_refused(gpu):
    rc, out = _run([os.path.join(BIN, "omr_client"), "-L", "2", "-H", "-M", "-n", str(1 << 20)])
    assert rc != 0 and "cannot be combined" in out, out


def test_server_client_rccl_one_worker(gpu):
    port = "19877"
    srv = subprocess.Popen([os.path.join(BIN, "omr_server"), "-p", port, "127.0.0.1"], stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True)
    try:
        rc, out = _run([os.path.join(BIN, "omr_client"), "-p", port, "-n", str(4 << 20), "-r", "0.095", "-W", "1",
                        "-R", "3", "-c", "-C", "127.0.0.1"])
        sout, _ = srv.communicate(timeout=60)
    finally:
        if srv.poll() is None:
            srv.kill()
    assert rc == 0, out
    assert "check OK" in out and "My ID is 0" in out
    assert srv.returncode == 0 and "test result is 0" in sout, sout


def _free_ports(k):
    import socket
    socks, ports = [], []
    for _ in range(k):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def _run_servers_clients(m, naggs, client_args, tmp_path, server_timeout=180):
    """naggs ./omr_server aggregator processes and m ./omr_client worker processes on one host and one GPU (HIP IPC
    transport); returns (server outputs, client outputs) after every process has exited."""
    ports = _free_ports(naggs)
    workers = ",".join(["127.0.0.1"] * m)
    aggs = ",".join(f"127.0.0.1:{p}" for p in ports)
    srvs = [subprocess.Popen([os.path.join(BIN, "omr_server"), "-p", str(p), "-G", "0", workers],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for p in ports]
    clis = [subprocess.Popen([os.path.join(BIN, "omr_client"), "-X", "ipc", "-l", str(w), "-G", "0"] +
                             [a.replace("{w}", str(w)) for a in client_args] + [aggs],
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for w in range(m)]
    outs = []
    try:
        for p in clis + srvs:
            outs.append(p.communicate(timeout=server_timeout)[0])
    finally:
        for p in clis + srvs:
            if p.poll() is None:
                p.kill()
    return [(p.returncode, o) for p, o in zip(srvs, outs[m:])], [(p.returncode, o) for p, o in zip(clis, outs[:m])]


@pytest.mark.parametrize("m,naggs", [(2, 1), (3, 2)])
def test_servers_are_aggregators_bulk(gpu, tmp_path, m, naggs):
    """./omr_server processes as the round's aggregator ranks (m workers + n servers, the reference's topology):
    every worker passes the working CHECK (client.cc:449-465) and reports the server count; each server reports
    its ID (server.cc:325)."""
    srv, cli = _run_servers_clients(m, naggs, ["-n", str(1 << 20), "-r", "0.3", "-W", "1", "-R", "3", "-c"],
                                    tmp_path)
    for w, (rc, out) in enumerate(cli):
        assert rc == 0 and "check OK" in out and "test result is 0" in out, out
        assert f"Number of aggregators: {naggs}; Number of workers is {m}; My ID is {w}" in out
    for j, (rc, out) in enumerate(srv):
        assert rc == 0 and "test result is 0" in out, out
        assert f"Number of aggregators: {naggs}; Number of workers is {m}; My ID is {j}" in out


def test_servers_clients_reference_round_count(gpu, tmp_path):
    """The reference's own warm-up / round counts (client.cc: 10 + 101 rounds) over the IPC transport, the CHECK on:
    every event of the transport is recorded far more often than the ~32 records one ROCm IPC event survives, so
    this pins the transport's event generations (csrc/omr_dist.hip, IpcDist)."""
    srv, cli = _run_servers_clients(2, 1, ["-n", str(1 << 20), "-r", "0.095", "-W", "10", "-R", "101", "-c"],
                                    tmp_path)
    for rc, out in cli + srv:
        assert rc == 0 and "test result is 0" in out, out
    for rc, out in cli:
        assert "check OK" in out, out


def _expected_trace(bufs, flags, n, B, L, naggs, worker):
    """The records worker `worker` sends and receives, in the client's -T order, from the oracle's literal state
    machines; aggregator of slot gs = 100 + gs % naggs (common.cc:381-383)."""
    ref = oracle.msg_simulate(bufs, flags, n, B, L.num_lanes, L.num_threads)
    exp = []
    for gs in range(L.num_threads * 16):
        agg = 100 + gs % naggs
        for rr in range(int(ref["rounds"][gs])):
            imm = int(ref["wimm"][worker, gs, rr])
            if imm:
                ln = imm >> 16
                exp.append((worker, agg, imm, ln, ref["wmsg"][worker, gs, rr, :ln * B + ln].tobytes()))
            imm = int(ref["rimm"][gs, rr])
            ln = imm >> 16
            exp.append((agg, worker, imm, ln, ref["rmsg"][gs, rr, :ln * B + ln].tobytes()))
    return exp


def _read_trace(path, B):
    data = open(path, "rb").read()
    got, pos = [], 0
    while pos < len(data):
        src, dst, imm, ln = np.frombuffer(data, dtype=np.uint32, count=4, offset=pos)
        pos += 16
        nbytes = (B * int(ln) + int(ln)) * 4
        got.append((int(src), int(dst), int(imm), int(ln), data[pos:pos + nbytes]))
        pos += nbytes
    return got


@pytest.mark.parametrize("m,naggs,B", [(3, 2, 256), (2, 1, 1024)])
def test_servers_are_aggregators_messages_trace(gpu, tmp_path, m, naggs, B):
    """-M with separate server processes: the workers and the servers exchange the reference's wire messages over
    the transport; each worker's -T trace (its messages and the replies it received) equals the oracle's per-slot
    state machines record for record, and every worker passes the CHECK."""
    n, r = 1 << 20, 0.2
    trace = str(tmp_path / "wire{w}.bin")
    srv, cli = _run_servers_clients(m, naggs, ["-M", "-n", str(n), "-b", str(B), "-r", str(r), "-W", "1", "-R", "2",
                                               "-c", "-T", trace], tmp_path)
    for rc, out in cli:
        assert rc == 0 and "check OK" in out, out
    for rc, out in srv:
        assert rc == 0 and "protocol rounds" in out, out
    L = Layout(n=n, block_size=B)
    bufs = [oracle.fill(oracle.gen_bitmap(w, r, L.nb), B) for w in range(m)]
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    for w in range(m):
        got = _read_trace(trace.replace("{w}", str(w)), B)
        exp = _expected_trace(bufs, flags, n, B, L, naggs, w)
        assert len(got) == len(exp), (w, len(got), len(exp))
        for i, (g, e) in enumerate(zip(got, exp)):
            assert g == e, f"worker {w} record {i}: {g[:4]} vs {e[:4]}"


def test_client_message_mode_trace(gpu, tmp_path):
    """./omr_client -L 3 -M: the round as the reference's messages; the -T wire trace (SURVEY.md Appendix B.6
    record layout) must equal, record for record and byte for byte, the oracle's literal state machines run on the
    reference generator's inputs (srand(myId+1), 0.01f blocks: client.cc:396-421)."""
    n, B, k, r = 1 << 20, 256, 3, 0.2
    trace = str(tmp_path / "wire.bin")
    rc, out = _run([os.path.join(BIN, "omr_client"), "-L", str(k), "-M", "-n", str(n), "-r", str(r), "-W", "1",
                    "-R", "2", "-c", "-T", trace])
    assert rc == 0, out
    assert "check OK" in out and "test result is 0" in out
    L = Layout(n=n, block_size=B)
    bufs = [oracle.fill(oracle.gen_bitmap(w, r, L.nb), B) for w in range(k)]
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    ref = oracle.msg_simulate(bufs, flags, n, B, L.num_lanes, L.num_threads)
    exp = []
    for gs in range(L.num_threads * 16):
        for rr in range(int(ref["rounds"][gs])):
            for w in range(k):
                imm = int(ref["wimm"][w, gs, rr])
                if imm:
                    ln = imm >> 16
                    exp.append((w, 100, imm, ln, ref["wmsg"][w, gs, rr, :ln * B + ln].tobytes()))
            imm = int(ref["rimm"][gs, rr])
            ln = imm >> 16
            for w in range(k):
                exp.append((100, w, imm, ln, ref["rmsg"][gs, rr, :ln * B + ln].tobytes()))
    data = open(trace, "rb").read()
    got, pos = [], 0
    while pos < len(data):
        src, dst, imm, ln = np.frombuffer(data, dtype=np.uint32, count=4, offset=pos)
        pos += 16
        nbytes = (B * int(ln) + int(ln)) * 4
        got.append((int(src), int(dst), int(imm), int(ln), data[pos:pos + nbytes]))
        pos += nbytes
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, f"record {i}: {g[:4]} vs {e[:4]}"


@pytest.mark.parametrize("extra", [[], ["--dist-sync"], ["--dist-pipe", "async"], ["--dist-mode", "allreduce"],
                                   ["--dist-mode", "dense"], ["--dist-pipe", "thread"]])
def test_bench_distributed_path_world1(gpu, extra):
    """bench.py's N>1 path as the driver launches it (torch.distributed.run, RCCL, the C++ round with two
    communicators, pipelined rounds joined before the closing sync), rehearsed at world 1."""
    import json
    root = os.path.dirname(PKG)
    # --standalone: the rendezvous store binds a free port itself (a port probed here can be taken before torchrun
    # binds it: EADDRINUSE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           "--nproc-per-node", "1", os.path.join(root, "bench.py"), "--force-dist", "--no-cpu",
           "--steps", "5", "--warmup", "2", "--size-mib", "64"] + extra
    rc, out = _run(cmd, timeout=240)
    assert rc == 0, "\n".join([ln for ln in out.splitlines() if "rc=" in ln or "Error" in ln][-20:]) + out[-1500:]
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["roofline"]["frac"] > 0
    assert "RCCL" in line["config"]["parallelism"]
    assert line["exchange"]["peers"] == 0 and line["exchange"]["ms_mean"] >= 0


@pytest.mark.parametrize("world,extra", [(2, []), (3, ["--dist-mode", "allreduce"]), (2, ["--dist-sync"]),
                                         (4, ["--dist-mode", "dense"]), (3, ["--dist-pipe", "thread"]),
                                         (8, []), (8, ["--dist-mode", "allreduce", "--dist-pipe", "thread"])])
def test_bench_distributed_path_ipc(gpu, world, extra):
    """bench.py's N>1 path with real exchanges on one GPU: torch.distributed.run with `world` ranks sharing the GPU
    over the HIP-IPC transport (gloo carries the id, barriers and the max-over-ranks time).  Rank 0's line reports
    the timed rounds' exchange with peers and non-zero bytes each way."""
    import json
    root = os.path.dirname(PKG)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--standalone", "--local-addr", "127.0.0.1", os.path.join(root, "bench.py"), "--force-dist",
           "--dist-transport", "ipc", "--no-cpu", "--steps", "12", "--warmup", "2", "--size-mib", "64",
           "--event-every", "3"] + extra
    rc, out = _run(cmd, timeout=240)
    assert rc == 0, "\n".join([ln for ln in out.splitlines() if "rc=" in ln or "Error" in ln][-20:]) + out[-1500:]
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    assert "HIP IPC" in line["config"]["parallelism"]
    x = line["exchange"]
    assert x["peers"] == world - 1 and x["timed_rounds"] >= 3 and x["ms_mean"] > 0
    assert x["bytes_out_per_rank"] > 0 and x["bytes_in_per_rank"] > 0


@pytest.mark.parametrize("world,mode", [(4, 1 | 0x100), (3, 0), (4, 2), (4, 1 | 0x400), (3, 0x400)])
def test_cpp_exchange_timing_loopback(gpu, world, mode):
    """OMR_ROUND_TIME_EXCHANGE: the timed round's result is unchanged, omr_ar_plan_exchange_time reports a
    duration and the exchange's bytes: out = this rank's sent blocks, and what the ranks send is what they
    receive; the dense stand-in moves (N-1)/N of the tensor each way."""
    B = 256
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), B, mode=1, seed=w + 3) for w in range(world)]
    board = D.omr_local_board_create(world)
    errs, res = [], [None] * world

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = torch.from_numpy(bufs[r].copy()).cuda()
            out = x.clone()
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            ms, bo, bi = ctypes.c_float(), ctypes.c_uint64(), ctypes.c_uint64()
            assert D.omr_ar_plan_exchange_time(plan, ctypes.byref(ms), None, None) == -1  # nothing timed yet (OMR_EINVAL)
            st = torch.cuda.Stream()
            sent = ctypes.c_uint64()
            assert D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), None, None, None, mode | 0x200,
                                          ctypes.byref(sent), None, st.cuda_stream) == 0, D.omr_dist_last_error()
            assert D.omr_ar_plan_join(plan, st.cuda_stream) == 0  # (a deferred round's exchange is issued here)
            assert D.omr_ar_plan_exchange_time(plan, ctypes.byref(ms), ctypes.byref(bo), ctypes.byref(bi)) == 0
            st.synchronize()
            res[r] = (ms.value, bo.value, bi.value, sent.value, out.cpu().numpy())
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    bounds = [s * L.rows // world for s in range(world + 1)]
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    for r in range(world):
        ms, bo, bi, sent, out = res[r]
        assert ms >= 0.0
        if (mode & 3) == 2:
            shard = (bounds[r + 1] - bounds[r]) * L.num_lanes * B * 4
            assert bo == bi == (world - 1) * shard
        else:
            assert bo == sent * B * 4 or (mode & 0x400)  # deferred: the call reports the previous round (none)
        full = bufs[r].copy()
        if (mode & 3) != 2:
            oracle.block_sum(bufs, L.n, B, L.num_lanes, 8, uf, full)
            exp = full if (mode & 3) == 0 else bufs[r].copy()
            if (mode & 3) == 1:
                lo, hi = bounds[r] * L.num_lanes * B, bounds[r + 1] * L.num_lanes * B
                exp[lo:hi] = full[lo:hi]
            assert (out.view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r}"
    if (mode & 3) != 2:
        assert sum(x[1] for x in res) == sum(x[2] for x in res)
