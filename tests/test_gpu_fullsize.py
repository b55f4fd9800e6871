"""BASELINE configs 4 and 5 at their own sizes, on one MI355X.

C4: 8 workers x 256 MiB fp32, -r 0.095 (seeds 1..8, the reference's 0.01f fill: client.cc:396-421):
  * the product's C++ multi-rank round (libomr_dist.so) with 8 loopback ranks sharing the GPU, reduce-scatter and
    all-reduce modes, synchronous and pipelined, and each rank's plan within 4x the tensor in device memory;
  * the m = 8 single-device sum k_scanm (omr_scan_sum_f32) over the same 8 tensors.
C5: 4 GiB fp32, -r 0.49, pinned host memory, staged (H2D/scan/D2H) and zero-copy host plans.

Checks (size-independent, no CPU pass over the data): flags == the generator bitmaps, each worker's next chain and
the aggregator's union chain == the oracle chains computed from the bitmaps (client.cc:19-31, server.cc:86-96),
every summed block == ka[count], where count is the number of workers that flag it and ka[k] is the k-fold
sequential fp32 sum of 0.01f from +0.0f (server.cc:97-98, :148-150; the reference CHECK's known answer,
client.cc:449-465)."""
import ctypes
import threading

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, ops

from test_cpp_dist import dist_lib

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

MODE_ALLREDUCE, MODE_RS, MODE_ASYNC, MODE_DEFER = 0, 1, 0x100, 0x400


def ka_table(m):
    """ka[k] = ((0.0f + 0.01f) + 0.01f) + ... k times, in fp32."""
    vals, acc = [np.float32(0.0)], np.float32(0.0)
    for _ in range(m):
        acc = np.float32(acc + np.float32(0.01))
        vals.append(acc)
    return np.array(vals, dtype=np.float32)


def expected_blocks(counts, ka, dev):
    """Per-block expected value ka[count], as a device tensor [nb]."""
    return torch.from_numpy(ka[counts]).to(dev)


def assert_blocks(out, exp_blk, L, sel=None):
    """out (device, n floats) viewed as [nb, B] equals exp_blk[b] in every element (bitwise), on rows `sel`."""
    ob = out.view(L.nb, L.block_size)
    eb = exp_blk[:, None].expand(L.nb, L.block_size)
    if sel is not None:
        ob, eb = ob[sel], eb[sel]
    assert torch.equal(ob.contiguous().view(torch.int32), eb.contiguous().view(torch.int32))


@pytest.fixture(scope="module")
def c4():
    L = Layout.from_bytes(256 << 20, 256)
    world = 8
    bms = [ops.gen_bitmap(w, 0.095, L.nb) for w in range(world)]  # srand(myId + 1), myId = w
    counts = np.sum(bms, axis=0).astype(np.int64)
    union = (counts > 0).astype(np.int32)
    nexts = [oracle.next_offsets(bm, L.n, 256, L.num_lanes, 8) for bm in bms]
    unext = oracle.next_offsets(union, L.n, 256, L.num_lanes, 8)
    return L, world, bms, counts, nexts, unext


@pytest.mark.parametrize("mode", [MODE_RS, MODE_ALLREDUCE, MODE_RS | MODE_DEFER, MODE_ALLREDUCE | MODE_ASYNC])
def test_c4_cpp_round_loopback(gpu, c4, mode):
    L, world, bms, counts, nexts, unext = c4
    D = dist_lib()
    board = D.omr_local_board_create(world)
    ka = ka_table(world)
    exp_blk = expected_blocks(counts, ka, gpu)
    errs, res, footprint = [], [None] * world, [0] * world
    rounds = 3

    def rank(r):
        try:
            torch.cuda.set_device(0)
            x = ops.fill_blocks(torch.from_numpy(bms[r]).to(gpu), L)
            out = x.clone()
            flags = torch.empty(L.nb, dtype=torch.int32, device=gpu)
            nxt = torch.empty(L.nb, dtype=torch.int32, device=gpu)
            unx = torch.empty(L.nb, dtype=torch.int32, device=gpu)
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, 256, L.num_lanes, 8, ctypes.byref(plan)) == 0
            footprint[r] = D.omr_ar_plan_device_bytes(plan)
            st = torch.cuda.Stream()
            for _ in range(rounds):  # x is never written; every round writes the same sums into out
                rc = D.omr_sparse_round_f32(plan, x.data_ptr(), out.data_ptr(), flags.data_ptr(), nxt.data_ptr(),
                                            unx.data_ptr(), mode, None, None, st.cuda_stream)
                assert rc == 0, D.omr_dist_last_error()
            assert D.omr_ar_plan_join(plan, st.cuda_stream) == 0
            st.synchronize()
            res[r] = (x, out, flags, nxt, unx)
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    D.omr_local_board_destroy(board)
    assert not errs, errs
    # the plan's device memory for 256 MiB at world 8 (round sets, three send buffers of 7/8 of the tensor, one
    # receive buffer): at most 4x the tensor (round 4 held about 9x)
    for r in range(world):
        assert 0 < footprint[r] <= 4 * L.nbytes, (r, footprint[r] / L.nbytes)
    bounds = [s * L.rows // world for s in range(world + 1)]
    rowsel = torch.arange(L.nb, device=gpu) // L.num_lanes
    for r in range(world):
        x, out, flags, nxt, unx = res[r]
        assert (flags.cpu().numpy() == bms[r]).all(), f"rank {r} flags"
        assert (nxt.cpu().numpy().view(np.uint32) == nexts[r]).all(), f"rank {r} next chain"
        assert (unx.cpu().numpy().view(np.uint32) == unext).all(), f"rank {r} union chain"
        if (mode & 0xff) == MODE_ALLREDUCE:
            assert_blocks(out, exp_blk, L)  # every worker holds the all-reduced tensor
        else:
            mine = (rowsel >= bounds[r]) & (rowsel < bounds[r + 1])
            assert_blocks(out, exp_blk, L, mine)  # its shard: the sums
            assert torch.equal(out.view(L.nb, 256)[~mine], x.view(L.nb, 256)[~mine])  # elsewhere: untouched


def test_c4_scanm_m8(gpu, c4):
    """k_scanm: the 8 workers' 256 MiB tensors summed on one device (omr_scan_sum_f32, m = 8)."""
    L, world, bms, counts, nexts, unext = c4
    bufs = [ops.fill_blocks(torch.from_numpy(bm).to(gpu), L) for bm in bms]
    out = torch.zeros(L.n, device=gpu)
    res = ops.ScanSumPlan(L, world, device=gpu).run(bufs, out)
    torch.cuda.synchronize()
    fl = res.flags.cpu().numpy()
    nx = res.next_offsets.cpu().numpy().view(np.uint32)
    for w in range(world):
        assert (fl[w] == bms[w]).all(), f"flags {w}"
        assert (nx[w] == nexts[w]).all(), f"next {w}"
    assert (nx[world] == unext).all(), "aggregator chain"
    assert_blocks(out, expected_blocks(counts, ka_table(world), gpu), L)


@pytest.mark.parametrize("zero_copy", [False, True])
def test_c5_host_resident_4gib(gpu, zero_copy):
    """4 GiB, -r 0.49, the gradient in pinned host memory (the reference's registered region, common.cc:873-914):
    staged (H2D row chunks -> in-place scan + aggregate -> D2H) or zero-copy (the kernel reads and writes the pinned
    buffer over PCIe).  The first element of every non-zero block is -0.0, which the aggregate 0.0f + x turns into
    +0.0 (server.cc:148-150, :97-98): the in-place result differs from the input exactly there."""
    L = Layout.from_bytes(4 << 30, 256)
    bm = ops.gen_bitmap(0, 0.49, L.nb)
    dev_x = ops.fill_blocks(torch.from_numpy(bm).to(gpu), L)
    nz = np.flatnonzero(bm)
    dev_x.view(L.nb, 256)[torch.from_numpy(nz).to(gpu), 0] = -0.0
    host = torch.empty(L.n, dtype=torch.float32).pin_memory()
    host.copy_(dev_x)
    exp = dev_x.view(L.nb, 256)
    exp[torch.from_numpy(nz).to(gpu), 0] = 0.0  # what the round must leave in the host buffer
    flags = torch.empty(L.nb, dtype=torch.int32).pin_memory()
    nxt = torch.empty(L.nb, dtype=torch.int32).pin_memory()
    plan = ops.HostPlan(L, chunk_rows=2048)
    secs = plan.run(host, flags, nxt, zero_copy=zero_copy)
    plan.close()
    assert secs > 0
    assert (flags.numpy() == bm).all()
    assert (nxt.numpy().view(np.uint32) == oracle.next_offsets(bm, L.n, 256, L.num_lanes, 8)).all()
    back = host.to(gpu)
    assert torch.equal(back.view(torch.int32), dev_x.view(torch.int32))
