"""GPU parity: the HIP path (through the C ABI) against the oracle and the golden fixtures.

Bar: flags, row masks, next offsets and block lists bit-exact; summed floats bit-exact against the oracle's
rank-order sum (server.cc:97-98 from a zeroed accumulator, server.cc:148-150) — tolerance 0 ulp here, because
the GPU adds the workers in the same rank order.  Full-size configs are checked through size-independent
properties (flags == the generator bitmap, next == the closed-form chain, out == the dense sum)."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, _lib, ops

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GOLDEN_NAMES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def u64(t):
    return t.cpu().numpy().view(np.uint64)


def run(bufs_np, L, out_init=None):
    dev = torch.device("cuda:0")
    bufs = [torch.from_numpy(b).to(dev) for b in bufs_np]
    out = torch.from_numpy(out_init.copy()).to(dev) if out_init is not None else torch.zeros(L.n, device=dev)
    res = ops.ScanSumPlan(L, len(bufs), device=dev).run(bufs, out)
    torch.cuda.synchronize()
    return res, out.cpu().numpy()


def oracle_all(bufs_np, L, out_init=None):
    B, NB, P = L.block_size, L.num_lanes, L.num_threads
    flags = [oracle.flags_from_data(b, B) for b in bufs_np]
    nexts = [oracle.next_offsets(f, L.n, B, NB, P) for f in flags]
    uf = oracle.union_flags(flags)
    unext = oracle.next_offsets(uf, L.n, B, NB, P)
    out = np.zeros(L.n, dtype=np.float32) if out_init is None else out_init.copy()
    oracle.block_sum(bufs_np, L.n, B, NB, P, uf, out)
    return flags, nexts, uf, unext, out


def assert_parity(bufs_np, L, out_init=None):
    res, out = run(bufs_np, L, out_init)
    flags, nexts, uf, unext, oout = oracle_all(bufs_np, L, out_init)
    m = len(bufs_np)
    gflags = res.flags.cpu().numpy()
    gmasks = u64(res.masks)
    gnext = u32(res.next_offsets)
    for w in range(m):
        assert (gflags[w] == flags[w]).all(), f"flags worker {w}"
        assert (gmasks[w] == oracle.row_masks(flags[w], L.num_lanes)).all(), f"masks worker {w}"
        assert (gnext[w] == nexts[w]).all(), f"next worker {w}"
    if m > 1:
        assert (gmasks[m] == oracle.row_masks(uf, L.num_lanes)).all(), "union masks"
        assert (gnext[m] == unext).all(), "aggregator chain"
    assert (out.view(np.uint32) == oout.view(np.uint32)).all(), "sum (bitwise)"
    return res, out


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_configs(gpu, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    L = Layout(n=meta["n"], block_size=meta["block_size"], num_threads=meta["parts"])
    m = meta["m"]
    bufs = [ops.make_worker_buffer(w, meta["density"], L, device=gpu) for w in range(m)]
    out = torch.zeros(L.n, device=gpu)
    res = ops.ScanSumPlan(L, m, device=gpu).run(bufs, out)
    torch.cuda.synchronize()
    flags = res.flags.cpu().numpy()
    nxt = u32(res.next_offsets)
    for w in range(m):
        assert (np.packbits(flags[w].astype(np.uint8), bitorder="little") == z["flags_w"][w]).all()
        assert (nxt[w] == z["next_w"][w]).all()
    if m > 1:
        assert (nxt[m] == z["union_next"]).all()
    o = out.cpu().numpy()
    assert hashlib.sha256(o.tobytes()).hexdigest() == meta["sum_sha256"]
    assert (o.reshape(L.nb, L.block_size) == z["ka_value"][z["counts"]][:, None]).all()  # CHECK known answer


def _rand_sparse(L, density, seed, m=1, values="hash"):
    bufs = []
    for w in range(m):
        bm = oracle.gen_bitmap(seed + w, density, L.nb)
        bufs.append(oracle.fill(bm, L.block_size, mode=1 if values == "hash" else 0, seed=seed + w))
    return bufs


@pytest.mark.parametrize("B", [256, 512, 1024])
@pytest.mark.parametrize("m", [1, 2, 3, 5, 8, 16])
def test_random_values_parity(gpu, B, m):
    L = Layout(n=1 << 20, block_size=B)
    assert_parity(_rand_sparse(L, 0.3, 11 * m + B, m), L)


@pytest.mark.parametrize("B,slots,m", [(256, 4, 2), (512, 4, 2), (256, 4, 5), (512, 4, 8), (1024, 8, 3)])
def test_narrow_rows_multi_worker(gpu, B, slots, m):
    """Rows narrower than k_scanm's default block group (16 lanes at B=256, 8 at B=512: layouts the C ABI admits) take
    the half-width group, so no group reaches into the next row; the last row is checked too."""
    L = Layout(n=1 << 19, block_size=B, num_slots=slots)
    assert L.num_lanes == slots * 1024 // B
    bufs = _rand_sparse(L, 0.4, 7 * m + B, m)
    for b in bufs:  # the last block of the tensor non-zero on every worker
        b[-B:] = 1.0
    assert_parity(bufs, L)


def test_all_zero(gpu):
    L = Layout(n=1 << 20)
    res, out = assert_parity([np.zeros(L.n, dtype=np.float32)], L)
    nxt = u32(res.next_offsets)[0]
    lanes = np.arange(L.nb) % L.num_lanes
    assert (nxt == L.sentinel + lanes * L.block_size).all()


def test_dense(gpu):
    L = Layout(n=1 << 20)
    assert_parity([np.full(L.n, 0.01, dtype=np.float32)], L)


def test_negative_zero_nan_subnormal(gpu):
    L = Layout(n=1 << 20)
    x = np.zeros(L.n, dtype=np.float32)
    B = L.block_size
    x[0 * B:1 * B] = -0.0                                   # head block of -0.0: flag 0, written back as +0.0
    x[70 * B:71 * B] = -0.0                                 # non-head -0.0 block: flag 0, untouched
    x[100 * B + 17] = np.nan                                # NaN counts as non-zero
    x[200 * B + 255] = np.float32(1e-45)                    # smallest subnormal
    x[300 * B:301 * B] = -0.0
    x[300 * B + 3] = 2.5                                    # mixed block: -0.0 elements become +0.0 (0.0 + -0.0)
    x[L.n - 1] = -3.0                                       # last element of the tensor
    init = np.full(L.n, -0.0, dtype=np.float32)             # untouched blocks keep -0.0
    res, out = assert_parity([x], L, out_init=init)
    f = res.flags.cpu().numpy()[0]
    assert f[0] == 0 and f[70] == 0 and f[100] == 1 and f[200] == 1 and f[300] == 1 and f[L.nb - 1] == 1


def test_negative_zero_sum_two_workers(gpu):
    L = Layout(n=1 << 20)
    a = _rand_sparse(L, 0.2, 5, 2)
    a[0][1000 * 256:1001 * 256] = -0.0
    a[1][1000 * 256 + 7] = 1.0
    assert_parity(a, L)


def test_config1_layout_short_partitions(gpu):
    """Config 1: 4 MiB, B=256, dense; 8 rows per partition (< one 64-row segment)."""
    L = Layout(n=1 << 20)
    assert L.rows_per_part == 8
    assert_parity(_rand_sparse(L, 1.0, 3), L)
    assert_parity(_rand_sparse(L, 0.0099, 3), L)


def test_single_partition_and_long_lanes(gpu):
    """NUM_THREADS=1 and long lane columns (look-ahead across many 64-row segments)."""
    L = Layout(n=16 << 20, block_size=1024, num_threads=1)
    assert_parity(_rand_sparse(L, 0.0005, 9), L)


def test_next_offsets_entry_point(gpu):
    L = Layout(n=4 << 20, block_size=256)
    bufs = _rand_sparse(L, 0.05, 21, 1)
    res, _ = run(bufs, L)
    nxt = ops.next_offsets(res.masks, L)
    torch.cuda.synchronize()
    assert (u32(nxt) == u32(res.next_offsets)).all()


def test_compact_gather_scatter_block_sum(gpu):
    L = Layout(n=4 << 20, block_size=256)
    bufs = _rand_sparse(L, 0.1, 31, 3)
    res, _ = run(bufs, L)
    uf = oracle.union_flags([oracle.flags_from_data(b, 256) for b in bufs])
    lst = ops.compact(res.masks[3], L)
    assert (lst.cpu().numpy() == np.nonzero(uf)[0]).all()
    # rows sub-range (an aggregator shard)
    r0, r1 = L.rows // 4, L.rows // 2
    part = ops.compact(res.masks[3], L, r0, r1).cpu().numpy()
    ref = np.nonzero(uf)[0]
    assert (part == ref[(ref >= r0 * 64) & (ref < r1 * 64)]).all()
    dev = torch.device("cuda:0")
    x = [torch.from_numpy(b).to(dev) for b in bufs]
    k = lst.numel()
    packed = torch.empty(k * 256, device=dev)
    ops.gather_blocks(x[1], lst, k, 256, packed)
    back = torch.zeros(L.n, device=dev)
    ops.scatter_blocks(packed, lst, k, 256, back)
    out = torch.zeros(L.n, device=dev)
    ops.block_sum(x, lst, k, 256, out)
    torch.cuda.synchronize()
    idx = lst.cpu().numpy()
    xb = bufs[1].reshape(-1, 256)
    assert (packed.cpu().numpy().reshape(-1, 256) == xb[idx]).all()
    bb = back.cpu().numpy().reshape(-1, 256)
    assert (bb[idx] == xb[idx]).all() and np.count_nonzero(np.delete(bb, idx, axis=0)) == 0
    oo = np.zeros(L.n, dtype=np.float32)
    oracle.block_sum(bufs, L.n, 256, 64, 8, uf, oo)
    ob = out.cpu().numpy().reshape(-1, 256)
    assert (ob[idx].view(np.uint32) == oo.reshape(-1, 256)[idx].view(np.uint32)).all()


def test_in_place_aliasing(gpu):
    """out may alias a worker buffer: the reference's in-place result (client.cc:89)."""
    L = Layout(n=1 << 20)
    bufs = _rand_sparse(L, 0.2, 41, 2)
    dev = torch.device("cuda:0")
    x = [torch.from_numpy(b).to(dev) for b in bufs]
    ops.ScanSumPlan(L, 2, device=dev).run(x, x[0])
    torch.cuda.synchronize()
    _, _, uf, _, oout = oracle_all(bufs, L, out_init=bufs[0])
    assert (x[0].cpu().numpy().view(np.uint32) == oout.view(np.uint32)).all()


@pytest.mark.slow
@pytest.mark.parametrize("nbytes,B,r", [(256 << 20, 256, 0.095), (1 << 30, 1024, 0.0099)])
def test_full_size_properties(gpu, nbytes, B, r):
    """Configs 2 and 3 at full size: flags == the reference generator's bitmap, next == the closed-form chain
    (oracle, from the bitmap), out == x on every written block (m = 1 sum of a single worker)."""
    L = Layout.from_bytes(nbytes, B)
    bm = ops.gen_bitmap(0, r, L.nb)
    x = ops.fill_blocks(torch.from_numpy(bm).to(gpu), L, mode=1, seed=1)
    out = torch.zeros(L.n, device=gpu)
    res = ops.ScanSumPlan(L, 1, device=gpu).run([x], out)
    torch.cuda.synchronize()
    assert (res.flags[0].cpu().numpy() == bm).all()
    assert (u32(res.next_offsets[0]) == oracle.next_offsets(bm, L.n, B, L.num_lanes, 8)).all()
    heads = (torch.arange(L.nb, device=gpu) // L.num_lanes) % L.rows_per_part == 0
    sel = torch.from_numpy(bm).to(gpu).bool() | heads
    xb, ob = x.view(L.nb, B), out.view(L.nb, B)
    assert torch.equal(ob[sel], xb[sel])
    assert int(torch.count_nonzero(ob[~sel])) == 0


@pytest.mark.parametrize("chunk_rows,zero_copy,B", [(7, False, 256), (64, False, 256), (4096, False, 256),
                                                    (512, True, 256), (512, True, 1024)])
def test_host_resident_pipeline(gpu, chunk_rows, zero_copy, B):
    """Pinned-host round: H2D chunks, in-place scan+aggregate, D2H (ragged last chunk with chunk_rows=7); or
    zero-copy, the single-pass kernel reading and writing the pinned buffer over PCIe (B=1024: K=2 segments)."""
    L = Layout(n=4 << 20, block_size=B)
    x = _rand_sparse(L, 0.3, 51)[0]
    x[5 * B:6 * B] = -0.0
    host = torch.from_numpy(x.copy()).pin_memory()
    flags = torch.empty(L.nb, dtype=torch.int32).pin_memory()
    nxt = torch.empty(L.nb, dtype=torch.int32).pin_memory()
    plan = ops.HostPlan(L, chunk_rows=chunk_rows)
    for _ in range(2 if zero_copy else 1):  # twice: the kernel's segment counters re-arm themselves
        host.copy_(torch.from_numpy(x))
        secs = plan.run(host, flags, nxt, zero_copy=zero_copy)
    plan.close()
    NB = L.num_lanes
    f = oracle.flags_from_data(x, B)
    exp = x.copy()
    oracle.block_sum([x], L.n, B, NB, 8, f, exp)
    assert secs > 0
    assert (flags.numpy() == f).all()
    assert (nxt.numpy().view(np.uint32) == oracle.next_offsets(f, L.n, B, NB, 8)).all()
    assert (host.numpy().view(np.uint32) == exp.view(np.uint32)).all()


def test_host_zero_copy_rejects_pageable(gpu):
    L = Layout(n=1 << 20, block_size=256)
    plan = ops.HostPlan(L)
    with pytest.raises(_lib.OmrError, match="not pinned"):
        plan.run(torch.zeros(L.n), zero_copy=True)
    plan.close()


@pytest.mark.parametrize("m,n", [(1, 4), (2, 1 << 20), (3, 12345 * 4), (8, (1 << 22) + 36), (16, 4096)])
def test_dense_sum(gpu, m, n):
    """omr_dense_sum_f32 (the dense stand-in aggregator): every element summed from +0.0f in rank order."""
    rng = np.random.default_rng(m * 7 + n)
    xs = [rng.standard_normal(n).astype(np.float32) for _ in range(m)]
    xs[0][:3] = -0.0
    exp = np.zeros(n, dtype=np.float32)
    for x in xs:
        exp = exp + x  # float32, sequential: ((0 + x0) + x1) + ...
    xd = [torch.from_numpy(x).to(gpu) for x in xs]
    out = torch.empty(n, dtype=torch.float32, device=gpu)
    ptrs = (ctypes.c_void_p * m)(*[t.data_ptr() for t in xd])
    assert _lib.load().omr_dense_sum_f32(ptrs, m, n, out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all()


# ------------------------------------------------------------------ single-pass fused kernel (k_scan1f)

def assert_fused_parity(x, L, out_init=None, reps=2):
    """Fused single launch vs the oracle; run twice so the self-resetting segment counters are exercised."""
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(x).to(dev)
    plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
    for _ in range(reps):
        out = torch.from_numpy(out_init.copy()).to(dev) if out_init is not None else torch.zeros(L.n, device=dev)
        res = plan.run([xd], out)
        torch.cuda.synchronize()
        f = oracle.flags_from_data(x, L.block_size)
        assert (res.flags[0].cpu().numpy() == f).all(), "flags"
        assert (u32(res.next_offsets[0]) == oracle.next_offsets(f, L.n, L.block_size, L.num_lanes,
                                                                L.num_threads)).all(), "next"
        exp = np.zeros(L.n, dtype=np.float32) if out_init is None else out_init.copy()
        oracle.block_sum([x], L.n, L.block_size, L.num_lanes, L.num_threads, f, exp)
        assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all(), "sum"
    ncols = L.num_threads * L.num_lanes  # the arrival counters lead the workspace; summaries are overwritten
    assert int(plan.workspace[: 4 * ncols].count_nonzero()) == 0, "segment counters must be left zeroed"


@pytest.mark.parametrize("n,B,parts,density", [
    (1 << 20, 256, 8, 0.3),        # config 1 layout: 8 rows per partition, K = 1, one partial batch
    (4 << 20, 256, 8, 0.095),      # K = 1, S = 32: two of 16 waves busy
    (16 << 20, 256, 8, 0.01),      # K = 1, S = 128
    (16 << 20, 1024, 8, 0.0099),   # 128 columns -> K = 2 segments of 64 rows
    (64 << 20, 1024, 8, 0.0099),   # K = 2 (config 3 split), S = 256
    (16 << 20, 1024, 1, 0.0005),   # one partition, 16 columns -> K = 16, long empty stretches
    (800 * 16384, 256, 8, 0.095),  # S = 100: seven busy waves, the last with a 4-row partial batch
    (20 << 20, 1024, 5, 0.2),      # 5 partitions of 256 rows, 80 columns -> K = 4, S = 64
    (8 << 20, 512, 8, 0.49),       # B = 512
    (4 << 20, 256, 8, 0.0),        # all zero: every chain is the sentinel
    (4 << 20, 256, 8, 1.0),        # dense
    # short segments (round 5): workgroups of 1, 2 or 4 waves, one per 16-row batch (k_scan1f's small-tensor shape)
    (8 << 20, 256, 8, 0.2),        # S = 64: 4-wave workgroups
    (1 << 20, 512, 8, 0.5),        # B = 512, S = 8: one wave
    (2 << 20, 1024, 8, 0.3),       # B = 1024, S = 16: 4-wave workgroups of 4-row batches
    (1 << 20, 256, 8, 1.0),        # config 1 itself, dense
])
def test_fused_parity(gpu, n, B, parts, density):
    L = Layout(n=n, block_size=B, num_threads=parts)
    x = oracle.fill(oracle.gen_bitmap(3, density, L.nb), B, mode=1, seed=5)
    assert_fused_parity(x, L)


def test_fused_edge_values(gpu):
    L = Layout(n=1 << 20)
    x = np.zeros(L.n, dtype=np.float32)
    B = L.block_size
    x[0:B] = -0.0
    x[64 * B + 9] = np.nan
    x[200 * B + 255] = np.float32(1e-45)
    x[L.n - 1] = -3.0
    assert_fused_parity(x, L, out_init=np.full(L.n, -0.0, dtype=np.float32))


MAX_N = 32767 * 8 * 16384  # the largest layout below the uint32 lane sentinel 4294934528 (client.cc:24): 16 GiB


@pytest.mark.slow
@pytest.mark.parametrize("nbytes,B,r", [(256 << 20, 256, 0.095), (1 << 30, 1024, 0.0099), (4 << 30, 256, 0.49),
                                        (MAX_N * 4, 256, 0.01), (MAX_N * 4, 1024, 0.01)])
def test_fused_full_size(gpu, nbytes, B, r):
    """Configs 2, 3 and 5 at full size, and the largest tensor whose offsets fit the reference's uint32 chains
    (odd rows per partition: ragged per-wave ranges; at B=1024 one segment per column): flags == the generator's
    bitmap, next == the oracle chain from it (offsets up to ~2^32), in-place result == input."""
    L = Layout(n=nbytes // 4, block_size=B)
    bm = ops.gen_bitmap(0, r, L.nb)
    x = ops.fill_blocks(torch.from_numpy(bm).to(gpu), L, mode=1, seed=1)
    ref = x.clone()
    plan = ops.ScanSumPlan(L, 1, device=gpu, fused=True)
    for _ in range(3):
        res = plan.run([x], x)  # in place, as the bench runs it
    torch.cuda.synchronize()
    assert (res.flags[0].cpu().numpy() == bm).all()
    assert (u32(res.next_offsets[0]) == oracle.next_offsets(bm, L.n, B, L.num_lanes, 8)).all()
    assert torch.equal(x, ref)  # 0.0f + x == x for these values: the in-place result is the input


@pytest.mark.parametrize("B,density", [(256, 0.095), (1024, 0.0099)])
def test_fused_bound_launch(gpu, B, density):
    """ScanSumPlan.bind (bench.py's per-step launch, arguments converted once): the same flags, next offsets and
    in-place sums as the oracle, over repeated launches on a side stream."""
    L = Layout(n=4 << 20, block_size=B)
    x_np = oracle.fill(oracle.gen_bitmap(2, density, L.nb), B, mode=1, seed=9)
    x = torch.from_numpy(x_np.copy()).to(gpu)
    plan = ops.ScanSumPlan(L, 1, device=gpu, fused=True)
    st = torch.cuda.Stream()
    launch = plan.bind(x, x, st)
    for _ in range(3):
        launch()
    st.synchronize()
    f = oracle.flags_from_data(x_np, B)
    assert (plan.flags[0].cpu().numpy() == f).all()
    assert (u32(plan.next_offsets[0]) == oracle.next_offsets(f, L.n, B, L.num_lanes, 8)).all()
    exp = x_np.copy()
    oracle.block_sum([x_np], L.n, B, L.num_lanes, 8, f, exp)
    assert (x.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all()
    with pytest.raises(ValueError):
        ops.ScanSumPlan(L, 2, device=gpu).bind(x, x)
