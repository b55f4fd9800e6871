"""GPU parity of the mask-addressed multi-rank round kernels, called through the C ABI (include/omr.h):
omr_worker_scan_f32 (scan + row masks), omr_round_plan / omr_round_plan_list (union / write set / prefixes / shard
counts, the aggregator bookkeeping of server.cc:83-96, and the aggregator chain in the same launch), omr_move_blocks_f32 (pack common.cc:405-407 / unpack client.cc:89)
and omr_shard_sum_f32 (server.cc:97-98 in rank order).  Checked against the oracle (flags, masks, next chains,
block sums) and plain numpy restatements of the index arithmetic.  Bar: bit-exact (integer work and rank-order
fp32 sums, 0 ulp)."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, _lib

pytestmark = pytest.mark.gpu


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def popc(a):
    a = a.astype(np.uint64)
    return np.array([bin(int(v)).count("1") for v in a.ravel()], dtype=np.int64).reshape(a.shape)


def np_prefix(masks):
    c = popc(masks)
    return np.concatenate([[0], np.cumsum(c)]).astype(np.uint32)


def np_write_set(masks, rpp, lanes):
    u = np.bitwise_or.reduce(masks, axis=0) if len(masks) else np.zeros(masks.shape[1], np.uint64)
    w = u.copy()
    allm = np.uint64((1 << lanes) - 1) if lanes < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    w[::rpp] |= allm
    return u, w


def set_blocks(mask_rows, lanes, r0=0, r1=None, skip=None):
    """Global block indices of the set bits of rows [r0, r1) in block order (optionally skipping a row range)."""
    r1 = len(mask_rows) if r1 is None else r1
    out = []
    for r in range(r0, r1):
        if skip is not None and skip[0] <= r < skip[1]:
            continue
        m = int(mask_rows[r])
        out += [r * lanes + l for l in range(lanes) if (m >> l) & 1]
    return np.array(out, dtype=np.int64)


@pytest.mark.parametrize("n,B,density", [(1 << 20, 256, 0.3), (4 << 20, 256, 0.095), (16 << 20, 1024, 0.0099),
                                         (8 << 20, 512, 0.49), (20 << 20, 1024, 0.2)])
def test_worker_scan_masks(gpu, n, B, density):
    L = Layout(n=n, block_size=B, num_threads=8 if n != 20 << 20 else 5)
    x = oracle.fill(oracle.gen_bitmap(2, density, L.nb), B, mode=1, seed=3)
    lib = _lib.load()
    xd = torch.from_numpy(x).to(gpu)
    flags = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    masks = torch.zeros(L.rows, dtype=torch.int64, device=gpu)
    wsb = lib.omr_scan_workspace_bytes(L.n, B, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=gpu)
    for _ in range(2):  # twice: the segment counters reset themselves; masks re-zeroed by the caller
        masks.zero_()
        assert lib.omr_worker_scan_f32(P(xd), L.n, B, L.num_lanes, L.num_threads, P(flags), P(nxt), P(masks), None,
                                       P(ws), wsb, stream()) == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        f = oracle.flags_from_data(x, B)
        assert (flags.cpu().numpy() == f).all()
        assert (masks.cpu().numpy().view(np.uint64) == oracle.row_masks(f, L.num_lanes)).all()
        assert (nxt.cpu().numpy().view(np.uint32) == oracle.next_offsets(f, L.n, B, L.num_lanes, L.num_threads)).all()
    assert torch.equal(xd, torch.from_numpy(x).to(gpu))  # out = NULL: the tensor is not written


def plan_ws(lib, gpu):
    """A zero-filled plan workspace (the kernel re-arms it after each launch)."""
    return torch.zeros(int(lib.omr_round_plan_workspace_words()), dtype=torch.int64, device=gpu)


def untag(counts, seq):
    """The (seq << 32) | count words of omr_round_plan: every one carries `seq`; returns the counts."""
    c = counts.cpu().numpy().view(np.uint64)
    assert ((c >> np.uint64(32)) == np.uint64(seq)).all(), (c >> np.uint64(32))
    return (c & np.uint64(0xFFFFFFFF)).astype(np.uint32)


@pytest.mark.parametrize("count,rows,rpp,lanes,stride_pad", [
    (1, 64, 8, 64, 0), (3, 512, 64, 64, 5), (8, 4096, 512, 64, 1024), (5, 1280, 256, 16, 0), (16, 100, 25, 32, 3),
    (2, 8192, 1024, 64, 0),                           # 32 chunks of one 256-row tile
    (7, 16384, 2048, 16, 0),                          # 64 chunks (the most)
    (3, 20480, 2560, 16, 0),                          # 40 chunks of two tiles
    (8, 300, 30, 64, 7),                              # a partial tile
    (16, 5000, 1000, 64, 0),                          # W = 16: 20 chunks, the last partial
    (4, 70000, 1000, 64, 0),                          # 55 chunks of five tiles, the last partial
])
def test_round_plan(gpu, count, rows, rpp, lanes, stride_pad):
    """omr_round_plan_list (round 5: row chunks side by side, ticketed, handing each other their popcount totals through
    the workspace; DPP wave scans) against numpy: union, write set, every array's prefix, the tagged counts at the shard
    bounds, the zeroed own masks and pack counters, and the aggregator chain, three launches in a row on one workspace;
    worker arrays at a stride whose tail (a position table) is not read as masks."""
    rng = np.random.default_rng(count * 31 + rows)
    stride = rows + stride_pad
    dens = rng.random(count) * 0.5
    masks = np.zeros((count, stride), dtype=np.uint64)
    lane_mask = np.uint64((1 << lanes) - 1 if lanes < 64 else (1 << 64) - 1)
    for c in range(count):
        bits = rng.random((rows, lanes)) < dens[c]
        masks[c, :rows] = (bits.astype(np.uint64) << np.arange(lanes, dtype=np.uint64)).sum(axis=1).astype(np.uint64)
        masks[c, :rows] &= lane_mask
        masks[c, rows:] = np.uint64(0xDEADBEEF)
    N = max(1, min(count, 8))
    bounds = np.array([s * rows // N for s in range(N + 1)], dtype=np.uint64)
    lib = _lib.load()
    md = torch.from_numpy(masks.reshape(-1).view(np.int64)).to(gpu)
    bd = torch.from_numpy(bounds.view(np.int64)).to(gpu)
    wset = torch.zeros(rows, dtype=torch.int64, device=gpu)
    umask = torch.zeros(rows, dtype=torch.int64, device=gpu)
    prefix = torch.zeros((count + 1) * (rows + 1), dtype=torch.int32, device=gpu)
    counts = torch.zeros((count + 1) * (N + 1), dtype=torch.int64, device=gpu)
    zero = torch.full((rows,), -1, dtype=torch.int64, device=gpu)
    zc = torch.full((8,), -1, dtype=torch.int32, device=gpu)
    ws = plan_ws(lib, gpu)
    B = 16384 // lanes
    unext = torch.full((rows * lanes,), -1, dtype=torch.int32, device=gpu)
    for seq in (7, 8, 9):
        prefix.zero_()
        umask.zero_()
        assert lib.omr_round_plan_list(P(md), count, stride, rows, rpp, lanes, P(bd), N + 1, P(wset),
                                       P(umask) if seq != 8 else None, P(prefix), P(counts), P(zero), P(zc), 8,
                                       P(ws), seq, P(unext), B, None, stream()) == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        untag(counts, seq)
        assert int(ws[0].item()) == 0  # the ticket counter re-armed
        if seq == 8:
            assert int(umask.count_nonzero()) == 0  # no union_masks asked for: not written
    mr = masks[:, :rows]
    u, w = np_write_set(mr, rpp, lanes)
    assert (umask.cpu().numpy().view(np.uint64) == u).all()
    assert (wset.cpu().numpy().view(np.uint64) == w).all()
    pre = prefix.cpu().numpy().view(np.uint32).reshape(count + 1, rows + 1)
    cn = untag(counts, 9).reshape(count + 1, N + 1)
    for a in range(count + 1):
        exp = np_prefix(mr[a] if a < count else w)
        assert (pre[a] == exp).all(), a
        assert (cn[a] == exp[bounds.astype(np.int64)]).all(), a
    assert int(zero.count_nonzero()) == 0 and int(zc.count_nonzero()) == 0
    flags = ((u[:, None] >> np.arange(lanes, dtype=np.uint64)) & np.uint64(1)).astype(np.int32).ravel()
    exp = oracle.next_offsets(flags, rows * lanes * B, B, lanes, rows // rpp)
    assert (unext.cpu().numpy().view(np.uint32) == exp).all()


def test_round_plan_counts_past_the_end(gpu):
    """Shard bounds that repeat (empty shards) and bounds at the end: every count = the prefix at its bound; a
    workspace reused across plans of different sizes (the chunk count changes) and a refused seq 0."""
    rows, lanes, rpp, count = 2048, 64, 256, 3
    rng = np.random.default_rng(5)
    masks = (rng.integers(0, 2 ** 63, size=(count, rows), dtype=np.int64)).view(np.uint64)
    bounds = np.array([0, 512, 512, 1500, 2048, 2048], dtype=np.uint64)
    lib = _lib.load()
    md = torch.from_numpy(masks.reshape(-1).view(np.int64)).to(gpu)
    bd = torch.from_numpy(bounds.view(np.int64)).to(gpu)
    wset = torch.zeros(rows, dtype=torch.int64, device=gpu)
    prefix = torch.zeros((count + 1) * (rows + 1), dtype=torch.int32, device=gpu)
    counts = torch.full(((count + 1) * len(bounds),), -1, dtype=torch.int64, device=gpu)
    ws = plan_ws(lib, gpu)
    assert lib.omr_round_plan(P(md), count, rows, rpp, lanes, P(bd), len(bounds), P(wset), None, P(prefix),
                              P(counts), None, P(ws), 0, stream()) != 0  # seq 0: refused
    _, w = np_write_set(masks, rpp, lanes)
    for seq, r in ((1, rows), (2, 512), (3, rows)):  # 8 chunks, then 2 on the same workspace, then 8
        b = np.minimum(bounds, r)
        bd = torch.from_numpy(b.view(np.int64)).to(gpu)
        assert lib.omr_round_plan_list(P(md), count, rows, r, rpp, lanes, P(bd), len(bounds), P(wset), None,
                                       P(prefix), P(counts), None, None, 0, P(ws), seq, None, 64, None,
                                       stream()) == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        cn = untag(counts, seq).reshape(count + 1, len(bounds))
        _, w = np_write_set(masks[:, :r], rpp, lanes)
        for a in range(count + 1):
            exp = np_prefix(masks[a, :r] if a < count else w)
            assert (cn[a] == exp[b.astype(np.int64)]).all(), (seq, a)


@pytest.mark.parametrize("count,rows,rpp,lanes", [(1, 64, 8, 64), (3, 512, 64, 64), (8, 4096, 512, 64),
                                                   (5, 1280, 256, 16), (16, 100, 25, 32), (3, 20480, 2560, 16)])
def test_round_plan_chain(gpu, count, rows, rpp, lanes):
    """omr_round_plan_list with union_next: the plan's outputs exactly as without it, plus the aggregator chain
    (server.cc:86-96, min_next over the workers) computed by the same launch from the workers' masks = the oracle's
    next offsets over the union of the workers' flags."""
    rng = np.random.default_rng(count * 7 + rows)
    B = 16384 // lanes
    masks = np.zeros((count, rows), dtype=np.uint64)
    for c in range(count):
        bits = rng.random((rows, lanes)) < rng.random() * 0.3
        masks[c] = (bits.astype(np.uint64) << np.arange(lanes, dtype=np.uint64)).sum(axis=1).astype(np.uint64)
    N = max(1, min(count, 8))
    bounds = np.array([s * rows // N for s in range(N + 1)], dtype=np.uint64)
    lib = _lib.load()
    md = torch.from_numpy(masks.view(np.int64)).to(gpu)
    bd = torch.from_numpy(bounds.view(np.int64)).to(gpu)
    ws = plan_ws(lib, gpu)
    outs = []
    for seq, chain in ((1, False), (2, True)):
        wset = torch.zeros(rows, dtype=torch.int64, device=gpu)
        umask = torch.zeros(rows, dtype=torch.int64, device=gpu)
        prefix = torch.zeros((count + 1) * (rows + 1), dtype=torch.int32, device=gpu)
        counts = torch.zeros((count + 1) * (N + 1), dtype=torch.int64, device=gpu)
        unext = torch.full((rows * lanes,), -1, dtype=torch.int32, device=gpu)
        assert lib.omr_round_plan_list(P(md), count, rows, rows, rpp, lanes, P(bd), N + 1, P(wset), P(umask),
                                       P(prefix), P(counts), None, None, 0, P(ws), seq, P(unext) if chain else None,
                                       B, None, stream()) == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        outs.append((wset.cpu(), umask.cpu(), prefix.cpu(), torch.from_numpy(untag(counts, seq)), unext.cpu()))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert torch.equal(a, b)
    assert (outs[0][4] == -1).all()  # no chain requested: union_next untouched
    u = np.bitwise_or.reduce(masks, axis=0)
    flags = ((u[:, None] >> np.arange(lanes, dtype=np.uint64)) & np.uint64(1)).astype(np.int32).ravel()
    exp = oracle.next_offsets(flags, rows * lanes * B, B, lanes, rows // rpp)
    assert (outs[1][4].numpy().view(np.uint32) == exp).all()


@pytest.mark.parametrize("B,rows,skip", [(256, 512, (0, 0)), (256, 512, (128, 256)), (512, 256, (200, 256)),
                                         (1024, 300, (0, 100)), (256, 64, (0, 64))])
def test_move_blocks_pack_unpack(gpu, B, rows, skip):
    lanes = 16384 // B
    rng = np.random.default_rng(rows + B)
    bits = rng.random((rows, lanes)) < 0.3
    masks = (bits.astype(np.uint64) << np.arange(lanes, dtype=np.uint64)).sum(axis=1).astype(np.uint64)
    pre = np_prefix(masks)
    n = rows * lanes * B
    x = rng.standard_normal(n).astype(np.float32)
    lib = _lib.load()
    xd = torch.from_numpy(x).to(gpu)
    md = torch.from_numpy(masks.view(np.int64)).to(gpu)
    pd = torch.from_numpy(pre.view(np.int32)).to(gpu)
    blocks = set_blocks(masks, lanes, skip=skip)
    packed = torch.full((max(len(blocks), 1) * B,), np.nan, dtype=torch.float32, device=gpu)
    assert lib.omr_move_blocks_f32(P(xd), P(packed), 0, P(md), P(pd), rows, lanes, B, skip[0], skip[1],
                                   stream()) == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    exp = x.reshape(-1, B)[blocks].ravel()
    assert (packed.cpu().numpy()[: len(exp)].view(np.uint32) == exp.view(np.uint32)).all()
    # unpack back into a fresh dense buffer: listed blocks restored, everything else untouched
    dense = torch.full((n,), -7.0, dtype=torch.float32, device=gpu)
    assert lib.omr_move_blocks_f32(P(packed), P(dense), 1, P(md), P(pd), rows, lanes, B, skip[0], skip[1],
                                   stream()) == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    want = np.full(n, -7.0, dtype=np.float32).reshape(-1, B)
    want[blocks] = x.reshape(-1, B)[blocks]
    assert (dense.cpu().numpy().view(np.uint32) == want.ravel().view(np.uint32)).all()


@pytest.mark.parametrize("count,me,B,packed_out,span", [
    (1, 0, 256, 0, None), (3, 1, 256, 0, None), (3, 2, 256, 1, None), (8, 5, 256, 1, None), (4, 0, 1024, 0, None),
    (2, 1, 512, 1, None), (16, 7, 256, 0, None),
    (3, 3, 256, 1, None),        # a dedicated aggregator (me == count): no own contribution
    (5, 2, 256, 0, (5, 70)),     # a row range that is not whole 32-row units (ragged shards)
    (4, 4, 512, 1, (1, 2)),      # one row
])
def test_shard_sum(gpu, count, me, B, packed_out, span):
    L = Layout(n=(2 << 20) if B == 256 else (4 << 20), block_size=B)
    lanes, rows = L.num_lanes, L.rows
    xs = [oracle.fill(oracle.gen_bitmap(c, 0.2, L.nb), B, mode=1, seed=11 + c) for c in range(count)]
    flags = [oracle.flags_from_data(x, B) for x in xs]
    masks = np.stack([oracle.row_masks(f, lanes) for f in flags])
    u, wset = np_write_set(masks, L.rows_per_part, lanes)
    N = 4
    r0, r1 = span if span else (rows // N, 3 * rows // N)  # default: a two-shard-wide row range
    # worker c != me sends its non-zero blocks of [r0, r1) in block order; streams concatenated in rank order
    streams, roff, acc = [], [], 0
    for c in range(count):
        roff.append(acc)
        if c != me:
            bl = set_blocks(masks[c], lanes, r0, r1)
            streams.append(xs[c].reshape(-1, B)[bl])
            acc += len(bl)
    recv = np.concatenate(streams).ravel() if streams and acc else np.zeros(B, np.float32)
    prefix = np.concatenate([np_prefix(masks[c]) for c in range(count)] + [np_prefix(wset)])
    lib = _lib.load()
    own = torch.from_numpy(xs[me] if me < count else np.zeros(L.n, np.float32)).to(gpu)
    recvd = torch.from_numpy(recv.astype(np.float32)).to(gpu)
    md = torch.from_numpy(masks.view(np.int64).ravel()).to(gpu)
    pd = torch.from_numpy(prefix.view(np.int32)).to(gpu)
    wd = torch.from_numpy(wset.view(np.int64)).to(gpu)
    roff_h = (ctypes.c_uint64 * count)(*roff)
    wblocks = set_blocks(wset, lanes, r0, r1)
    if packed_out:
        out = torch.full((len(wblocks) * B,), np.nan, dtype=torch.float32, device=gpu)
    else:
        out = own.clone()  # dense, in place semantics: other blocks keep x_me
    assert lib.omr_shard_sum_f32(P(own) if me < count else None, me, P(recvd), roff_h, P(md), count, P(pd), P(wd),
                                 rows, r0, r1, lanes, B, packed_out, P(out), stream()) == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    # expected: rank-order sums from +0.0 over the workers that flag the block (server.cc:97-98, :148-150)
    exp_blocks = np.zeros((len(wblocks), B), dtype=np.float32)
    for i, b in enumerate(wblocks):
        s = np.zeros(B, dtype=np.float32)
        for c in range(count):
            if flags[c][b]:
                s = (s + xs[c].reshape(-1, B)[b]).astype(np.float32)
        exp_blocks[i] = s
    got = out.cpu().numpy()
    if packed_out:
        assert (got.view(np.uint32) == exp_blocks.ravel().view(np.uint32)).all()
    else:
        want = (xs[me].copy() if me < count else np.zeros(L.n, np.float32)).reshape(-1, B)
        want[wblocks] = exp_blocks
        assert (got.view(np.uint32) == want.ravel().view(np.uint32)).all()


# ---------------------------------------------------------------- the round check (round 6)

@pytest.mark.parametrize("n,B,density,pack", [(4 << 20, 256, 0.095, False), (16 << 20, 1024, 0.0099, False),
                                              (8 << 20, 256, 0.3, True), (64 << 20, 256, 0.095, True)])
def test_round_check_slots(gpu, n, B, density, pack):
    """omr_worker_scan_check_f32 / omr_worker_scan_pack_check_f32: one slot per scan workgroup, (seq << 32) | its
    non-zero blocks; the slots add up to the masks' popcount, the oracle's non-zero block count.  The completion word:
    done[1] = seq after each launch, done[0] back at zero."""
    L = Layout(n=n, block_size=B)
    x = oracle.fill(oracle.gen_bitmap(4, density, L.nb), B, mode=1, seed=9)
    f = oracle.flags_from_data(x, B)
    lib = _lib.load()
    ns = int(lib.omr_round_check_slots(L.n, B, L.num_lanes, L.num_threads))
    assert ns == int(lib.omr_tally_slots(L.n, B, L.num_lanes, L.num_threads)) > 0
    xd = torch.from_numpy(x).to(gpu)
    flags = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    masks = torch.zeros(L.rows, dtype=torch.int64, device=gpu)
    slots = torch.zeros(ns, dtype=torch.int64, device=gpu)
    wsb = lib.omr_scan_workspace_bytes(L.n, B, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=gpu)
    done = torch.zeros(2, dtype=torch.int32, device=gpu)
    for seq in (7, 8):
        masks.zero_()
        if pack:
            bounds = np.array([0, L.rows // 2, L.rows], dtype=np.uint64)
            ent = ctypes.c_uint64()
            assert lib.omr_pack_geometry(L.n, B, L.num_lanes, L.num_threads, None, None, ctypes.byref(ent)) == 0
            send = torch.zeros(L.n, dtype=torch.float32, device=gpu)
            cnt = torch.zeros(2, dtype=torch.int32, device=gpu)
            pos = torch.zeros(int(ent.value), dtype=torch.int32, device=gpu)
            rc = lib.omr_worker_scan_pack_check_f32(P(xd), L.n, B, L.num_lanes, L.num_threads, P(flags), P(nxt),
                                                    P(masks), None, bounds.ctypes.data, 2, 0, P(send), P(cnt), P(pos),
                                                    P(ws), wsb, P(slots), seq, P(done), stream())
        else:
            rc = lib.omr_worker_scan_check_f32(P(xd), L.n, B, L.num_lanes, L.num_threads, P(flags), P(nxt), P(masks),
                                               None, P(ws), wsb, P(slots), seq, P(done), stream())
        assert rc == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        assert done.cpu().tolist() == [0, seq]
        s = slots.cpu().numpy().view(np.uint64)
        assert ((s >> np.uint64(32)) == np.uint64(seq)).all()
        assert int((s & np.uint64(0xFFFFFFFF)).sum()) == int(f.sum()) == int(popc(masks.cpu().numpy()).sum())
        assert (masks.cpu().numpy().view(np.uint64) == oracle.row_masks(f, L.num_lanes)).all()


def test_round_plan_check(gpu):
    """omr_round_plan_check: status (seq << 32) | 0 on the workers' own arrays; | 0x100 + c when a slot of worker c
    carries another round's number (its array read before its scan wrote it); | 0x200 + c when worker c's masks hold
    fewer bits than its slots count (read before its scan finished).  The plan's other outputs are unchanged."""
    B, m = 256, 3
    L = Layout(n=4 << 20, block_size=B)
    lib = _lib.load()
    ns = int(lib.omr_round_check_slots(L.n, B, L.num_lanes, L.num_threads))
    stride = L.rows + ns + 3
    arrays = torch.zeros(m, stride, dtype=torch.int64, device=gpu)
    wsb = lib.omr_scan_workspace_bytes(L.n, B, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=gpu)
    flags = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    seq = 41
    fl = []
    for c in range(m):
        x = oracle.fill(oracle.gen_bitmap(c, 0.2, L.nb), B, mode=1, seed=c)
        fl.append(oracle.flags_from_data(x, B))
        xd = torch.from_numpy(x).to(gpu)
        row = arrays[c]
        assert lib.omr_worker_scan_check_f32(P(xd), L.n, B, L.num_lanes, L.num_threads, P(flags), P(nxt),
                                             ctypes.c_void_p(row.data_ptr()), None, P(ws), wsb,
                                             ctypes.c_void_p(row.data_ptr() + 8 * (L.rows + 3)), seq, None,
                                             stream()) == 0
    torch.cuda.synchronize()
    pws = plan_ws(lib, gpu)
    bounds = torch.tensor([0, L.rows // 2, L.rows], dtype=torch.int64, device=gpu)
    wset = torch.zeros(L.rows, dtype=torch.int64, device=gpu)
    prefix = torch.zeros((m + 1) * (L.rows + 1), dtype=torch.int32, device=gpu)
    counts = torch.zeros((m + 1) * 3, dtype=torch.int64, device=gpu)
    status = torch.zeros(1, dtype=torch.int64, device=gpu)

    def plan(s):
        # (a fresh workspace per launch: the arrays' slots carry `seq`, so the launches here repeat it, which the plan's
        # contract forbids on one workspace -- its chunks' tagged totals of the previous launch would pass as this one's)
        pws = plan_ws(lib, gpu)
        assert lib.omr_round_plan_check(P(arrays), m, stride, L.rows, L.rows_per_part, L.num_lanes, P(bounds), 3,
                                        P(wset), None, P(prefix), P(counts), None, None, 0, P(pws), s, None, B, None,
                                        L.rows + 3, ns, P(status), stream()) == 0, lib.omr_last_error()
        torch.cuda.synchronize()
        v = int(status.cpu().numpy().view(np.uint64)[0])
        assert v >> 32 == s
        return v & 0xFFFFFFFF

    assert plan(seq) == 0
    masks = arrays[:, :L.rows].cpu().numpy().view(np.uint64)
    exp_c = np.array([[np_prefix(masks[a])[b] for b in (0, L.rows // 2, L.rows)] for a in range(m)])
    assert (untag(counts, seq).reshape(m + 1, 3)[:m] == exp_c).all()
    # the same arrays checked as another round's: every slot is stale (the first worker found is reported)
    assert plan(seq + 1) & 0xF00 == 0x100
    # worker 2's last slot from an earlier round
    sl = arrays[2, L.rows + 3 + ns - 1].item()
    arrays[2, L.rows + 3 + ns - 1] = ((seq - 4) << 32) | (sl & 0xFFFFFFFF)
    assert plan(seq) == 0x100 | 2
    arrays[2, L.rows + 3 + ns - 1] = sl
    assert plan(seq) == 0
    # worker 1's masks missing a row's bits (a copy that overtook its scan)
    r = int(np.nonzero(masks[1])[0][5])
    arrays[1, r] = 0
    assert plan(seq) == 0x200 | 1
