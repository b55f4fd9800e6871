"""A failed exchange must leave the transport usable: omr_dist_inject_fault makes the next
exchange fail after a chosen number of pieces.

* RCCL, one-rank communicator in this process: the failing exchange opened an ncclGroupStart; the group must be closed
  on the error path, or the next all-gather would be captured by the open group and never launched (the data would
  not move).  Checked: the exchange returns an error, the next all-gather moves its bytes, and a full round then
  matches the oracle.
* Loopback, two ranks as threads: a round whose exchange fails (on both ranks, or on one rank after its first piece)
  returns the error on the failing rank(s) without leaving the peer waiting; the next round on the same plans is
  bit-exact against the oracle (synchronous and deferred rounds)."""
import ctypes
import threading

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, cdist

from test_cpp_dist import dist_lib

pytestmark = pytest.mark.gpu


def test_rccl_failed_exchange_closes_group(gpu):
    L = Layout(n=1 << 20, block_size=256)
    eng = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        eng.inject_fault(0)
        assert eng.exchange([None], [None]) != 0  # failed inside the RCCL group
        src = torch.arange(64, dtype=torch.int32, device=gpu)
        dst = torch.zeros(64, dtype=torch.int32, device=gpu)
        eng.allgather(src, dst)  # launched only if the failed exchange closed its group
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
        assert eng.exchange([None], [None]) == 0  # the fault fires once
        # a whole round (reduce-scatter at world 1: the shard is the whole tensor) then matches the oracle
        x = oracle.fill(oracle.gen_bitmap(0, 0.2, L.nb), 256, mode=1, seed=5)
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
    finally:
        eng.close()


@pytest.mark.parametrize("fault_ranks,after,mode", [
    ((0, 1), 0, 0),      # both ranks fail before their first piece, all-reduce
    ((0,), 1, 1),        # rank 0 fails after its only piece (after the copy), reduce-scatter
    ((1,), 0, 0x401),    # deferred reduce-scatter rounds: the failing exchange is issued by a later call
])
def test_loopback_failed_exchange_then_rounds(gpu, fault_ranks, after, mode):
    world, B = 2, 256
    L = Layout(n=2 << 20, block_size=B)
    D = dist_lib()
    D.omr_dist_inject_fault.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    bufs = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), B, mode=1, seed=w + 11) for w in range(world)]
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    board = D.omr_local_board_create(world)
    errs, outs, rcs = [], [None] * world, [[] for _ in range(world)]
    defer = (mode & 0x400) != 0

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = torch.from_numpy(bufs[r].copy()).cuda()
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, B, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            if r in fault_ranks:
                assert D.omr_dist_inject_fault(d, after) == 0
            out = x.clone()
            if defer:  # three deferred rounds: the first call's exchange is issued by the third call and fails
                res = [x.clone() for _ in range(3)]
                for k in range(3):
                    rcs[r].append(D.omr_sparse_round_f32(plan, x.data_ptr(), res[k].data_ptr(), None, None, None,
                                                         mode, None, None, st.cuda_stream))
                rcs[r].append(D.omr_ar_plan_join(plan, st.cuda_stream))
            else:
                rcs[r].append(D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), None, None, None, mode,
                                                     None, None, st.cuda_stream))
            st.synchronize()
            out = x.clone()  # a fresh round on the same plan and transport
            rc = D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), None, None, None, mode & 0xFF, None, None,
                                        st.cuda_stream)
            assert rc == 0, D.omr_dist_last_error()
            st.synchronize()
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
    for r in range(world):
        assert any(rc != 0 for rc in rcs[r]) == (r in fault_ranks), (r, rcs[r])
    bounds = [s * L.rows // world for s in range(world + 1)]
    rowf = L.num_lanes * B
    for r in range(world):
        exp = bufs[r].copy()
        full = bufs[r].copy()
        oracle.block_sum(bufs, L.n, B, L.num_lanes, 8, uf, full)
        if (mode & 0xFF) == 1:  # reduce-scatter: only this rank's shard rows carry the sums
            exp[bounds[r] * rowf:bounds[r + 1] * rowf] = full[bounds[r] * rowf:bounds[r + 1] * rowf]
        else:
            exp = full
        assert (outs[r].view(np.uint32) == exp.view(np.uint32)).all(), f"rank {r}"
