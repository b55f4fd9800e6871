"""The round's fused pack and the shard sum over its column streams, through the C ABI, against the oracle.

omr_worker_scan_pack_f32 (the worker scan with the pack of common.cc:399-407 fused in): besides flags, next offsets
and row masks (client.cc:19-31), every non-zero block of a row of another shard is written to that shard's send
stream (the streams in shard order, the own shard's left out: omr_pack_send_offset); the stream's length is its
counter, and the position table locates every block (segment, 64-row group, lane) -> stream place.  Checked: each stream is a permutation of exactly its shard's non-zero blocks, every block sits
where the table says, nothing outside the streams is written, own-shard rows are not packed; including densities
that overflow the waves' LDS slots (the re-read path), B = 512 / 1024 (two column segments per partition), and 1-8
shards.

omr_shard_sum_list_f32 (server.cc:83-99 over those streams): M workers' scans on one device, their streams
concatenated as the transport would deliver them to an aggregator, the bookkeeping from omr_round_plan_list over the
all-gathered masks + tables, the pair list built by the plan launch and by a launch of its own, then the shard sums —
dense in place and packed in write-set order — bit-exact against the oracle's rank-order sum (0 ulp)."""
import ctypes

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, _lib

pytestmark = pytest.mark.gpu
SENT = np.float32(1234.5)


def P(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def geometry(L):
    lib = _lib.load()
    S, gps, ent = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    assert lib.omr_pack_geometry(L.n, L.block_size, L.num_lanes, L.num_threads, ctypes.byref(S), ctypes.byref(gps),
                                 ctypes.byref(ent)) == 0
    return S.value, gps.value, ent.value


def bounds_of(L, world):
    return np.array([s * L.rows // world for s in range(world + 1)], dtype=np.uint64)


def send_offset(L, bounds, own, s):
    """Where shard s's stream starts in the send buffer (floats): omr_pack_send_offset, checked against its rule."""
    lib = _lib.load()
    bh = bounds.astype(np.uint64)
    tot = ctypes.c_uint64()
    off = lib.omr_pack_send_offset(bh.ctypes.data_as(ctypes.c_void_p), len(bounds) - 1, own, s, L.num_lanes,
                                   L.block_size, ctypes.byref(tot))
    rowf = L.num_lanes * L.block_size
    own_rows = int(bounds[own + 1] - bounds[own]) if own >= 0 else 0
    assert off == (int(bounds[s]) - (own_rows if 0 <= own < s else 0)) * rowf
    assert tot.value == L.n - own_rows * rowf
    return off


def scan_pack(xd, L, bounds, own, masks_out=None, table_out=None):
    """One omr_worker_scan_pack_f32 call; returns (flags, next, masks, send, counters, table) on the host."""
    lib = _lib.load()
    dev = xd.device
    S, gps, ent = geometry(L)
    world = len(bounds) - 1
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    masks = masks_out if masks_out is not None else torch.zeros(L.rows, dtype=torch.int64, device=dev)
    send = torch.full((L.n,), float(SENT), device=dev)
    cnt = torch.zeros(world, dtype=torch.int32, device=dev)
    table = table_out if table_out is not None else torch.full((ent,), -1, dtype=torch.int32, device=dev)
    wsb = lib.omr_scan_workspace_bytes(L.n, L.block_size, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    bh = bounds.astype(np.uint64)
    rc = lib.omr_worker_scan_pack_f32(P(xd), L.n, L.block_size, L.num_lanes, L.num_threads, P(flags), P(nxt),
                                      P(masks), None, bh.ctypes.data_as(ctypes.c_void_p), world, own, P(send), P(cnt),
                                      P(table), P(ws), wsb, stream())
    assert rc == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    return (flags.cpu().numpy(), nxt.cpu().numpy().view(np.uint32), masks.cpu().numpy().view(np.uint64),
            send.cpu().numpy(), cnt.cpu().numpy().view(np.uint32), table.cpu().numpy().view(np.uint32))


def stream_positions(f, L, S, gps, table, r0, r1):
    """(block, stream position) of every flagged block of rows [r0, r1), from the table + the column's bits."""
    NB = L.num_lanes
    fl = f.reshape(L.rows, NB)
    out = []
    for r in range(r0, r1):
        for ln in np.nonzero(fl[r])[0]:
            seg, j = r // S, (r % S) // 64
            g0 = seg * S + j * 64
            below = int(fl[g0:r, ln].sum())
            out.append((r * NB + int(ln), int(table[(seg * gps + j) * NB + ln]) + below))
    return out


@pytest.mark.parametrize("n,B,density,world,own", [
    (2 << 20, 256, 0.095, 2, 0),
    (2 << 20, 256, 0.3, 4, 3),
    (4 << 20, 256, 0.9, 8, 5),      # beyond the waves' LDS slots: the lowest non-zero rows are re-read
    (4 << 20, 512, 0.2, 4, -1),     # a worker that aggregates none packs every shard
    (16 << 20, 1024, 0.05, 2, 1),   # two column segments per partition (K = 2)
    (16 << 20, 1024, 1.0, 8, 0),    # dense at B = 1024: 2 stash slots per wave, the rest re-read
    (64 << 20, 256, 0.095, 8, 2),   # config 4's layout at 256 MiB (512-row segments, 8 groups each)
])
def test_worker_scan_pack(gpu, n, B, density, world, own):
    L = Layout(n=n, block_size=B)
    S, gps, ent = geometry(L)
    bounds = bounds_of(L, world)
    lib = _lib.load()
    assert lib.omr_pack_supported(L.n, B, L.num_lanes, L.num_threads, bounds.ctypes.data_as(ctypes.c_void_p),
                                  world) == 0, lib.omr_last_error()
    x = oracle.fill(oracle.gen_bitmap(3, density, L.nb), B, mode=1, seed=9)
    xd = torch.from_numpy(x).to(gpu)
    f = oracle.flags_from_data(x, B)
    for _ in range(2):  # twice: the workspace counters reset themselves; the pack counters start at zero each call
        flags, nxt, masks, send, cnt, table = scan_pack(xd, L, bounds, own)
        assert (flags == f).all()
        assert (masks == oracle.row_masks(f, L.num_lanes)).all()
        assert (nxt == oracle.next_offsets(f, L.n, B, L.num_lanes, L.num_threads)).all()
        rowf = L.num_lanes * B
        touched = np.zeros(L.n, dtype=bool)
        for s in range(world):
            r0, r1 = int(bounds[s]), int(bounds[s + 1])
            nz = int(f.reshape(L.rows, -1)[r0:r1].sum())
            if s == own:
                assert cnt[s] == 0
                continue
            assert cnt[s] == nz, (s, cnt[s], nz)
            pos = stream_positions(f, L, S, gps, table, r0, r1)
            places = sorted(p for _, p in pos)
            assert places == list(range(nz)), f"shard {s}: stream places are not a permutation of 0..{nz}"
            base = send_offset(L, bounds, own, s)
            for blk, p in pos:
                got = send[base + p * B:base + (p + 1) * B]
                assert (got.view(np.uint32) == x[blk * B:(blk + 1) * B].view(np.uint32)).all(), (s, blk, p)
            touched[base:base + nz * B] = True
        assert (send[~touched] == SENT).all(), "a store outside the shard streams"


def test_pack_rejects_ragged_shards(gpu):
    L = Layout(n=2 << 20, block_size=256)
    lib = _lib.load()
    b = bounds_of(L, 3)  # 128 rows over 3 shards: 42 / 85, not whole 16-row segments
    assert lib.omr_pack_supported(L.n, 256, L.num_lanes, L.num_threads, b.ctypes.data_as(ctypes.c_void_p), 3) != 0
    assert b"segment" in lib.omr_last_error()


@pytest.mark.parametrize("n,B,density,m,naggs,colocated", [
    (2 << 20, 256, 0.2, 2, 2, True),
    (4 << 20, 256, 0.095, 8, 8, True),
    (4 << 20, 256, 0.6, 4, 4, True),    # stash overflow on every worker
    (4 << 20, 512, 0.3, 3, 2, False),   # dedicated aggregators: the workers pack every shard
    (16 << 20, 1024, 0.1, 4, 4, True),
    (2 << 20, 256, 0.5, 16, 8, False),  # the largest group (OMR_MAX_WORKERS workers)
])
@pytest.mark.parametrize("packed_out", [0, 1])
def test_shard_sum_list(gpu, n, B, density, m, naggs, colocated, packed_out):
    L = Layout(n=n, block_size=B)
    lib = _lib.load()
    S, gps, ent = geometry(L)
    rows = L.rows
    mstride = rows + (ent + 1) // 2
    bounds = bounds_of(L, naggs)
    bufs = [oracle.fill(oracle.gen_bitmap(w + 20, density, L.nb), B, mode=1, seed=w + 5) for w in range(m)]
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    uf = oracle.union_flags(flags)
    full = np.zeros(L.n, dtype=np.float32)
    oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, full)
    # every worker's scan + pack; masks and table land in its slot of the all-gathered array
    masks_all = torch.zeros(m * mstride, dtype=torch.int64, device=gpu)
    xds = [torch.from_numpy(b).to(gpu) for b in bufs]
    sends = []
    for w in range(m):
        own = w if colocated else -1
        slot = masks_all[w * mstride:(w + 1) * mstride]
        tbl = slot[rows:].view(torch.int32)[:ent]
        res = scan_pack(xds[w], L, bounds, own, masks_out=slot[:rows], table_out=tbl)
        sends.append((res[3], res[4]))
    # the bookkeeping over the all-gathered arrays (stride mstride)
    wset = torch.zeros(rows, dtype=torch.int64, device=gpu)
    umask = torch.zeros(rows, dtype=torch.int64, device=gpu)
    prefix = torch.zeros((m + 1) * (rows + 1), dtype=torch.int32, device=gpu)
    bdev = torch.from_numpy(bounds.astype(np.int64)).to(gpu)
    counts = torch.zeros((m + 1) * (naggs + 1), dtype=torch.int64, device=gpu)
    ws = torch.zeros(int(lib.omr_round_plan_workspace_words()), dtype=torch.int64, device=gpu)
    seq = 1
    rc = lib.omr_round_plan_list(P(masks_all), m, mstride, rows, L.rows_per_part, L.num_lanes, P(bdev), naggs + 1,
                                 P(wset), P(umask), P(prefix), P(counts), None, None, 0, P(ws), seq, None, B, None,
                                 stream())
    assert rc == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    ws_np = wset.cpu().numpy().view(np.uint64)
    rowf = L.num_lanes * B
    for s in range(naggs):
        me = s if colocated else m  # the co-located aggregator of shard s is worker s
        r0, r1 = int(bounds[s]), int(bounds[s + 1])
        # what the transport delivers: every other worker's stream of shard s, peer by peer
        parts, offs, k = [], np.zeros(m, dtype=np.uint64), 0
        for w in range(m):
            if w == me:
                continue
            send, cnt = sends[w]
            offs[w] = k
            base = send_offset(L, bounds, w if colocated else -1, s)
            parts.append(send[base:base + int(cnt[s]) * B])
            k += int(cnt[s])
        recv = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(B, np.float32)).to(gpu)
        if packed_out:
            out = torch.zeros(L.n, device=gpu)
        else:
            out = xds[me].clone() if colocated else torch.zeros(L.n, device=gpu)
        own = xds[me] if colocated else None
        out0 = out.clone()
        # the pair list, built by the plan launch (omr_round_plan_list) and in a launch of its own
        # (omr_sum_list_build); the sums over each must equal the oracle's bit for bit, and each other
        units, cap = ctypes.c_uint64(), ctypes.c_uint32()
        outs = []
        assert lib.omr_sum_list_geometry(L.n, B, L.num_lanes, L.num_threads, r0, r1, m, ctypes.byref(units),
                                         ctypes.byref(cap)) == 0, lib.omr_last_error()
        for how in ("plan", "build"):
            rec = torch.full((max(1, units.value * cap.value),), -1, dtype=torch.int64, device=gpu)
            cnt = torch.full((max(1, units.value),), 7, dtype=torch.int32, device=gpu)
            sl = _lib.SumList(P(rec), P(cnt), r0, r1, 2 * rows, me)
            for w in range(m):
                sl.recv_offsets[w] = int(offs[w])
            if how == "plan":
                seq += 1
                rc = lib.omr_round_plan_list(P(masks_all), m, mstride, rows, L.rows_per_part, L.num_lanes, P(bdev),
                                             naggs + 1, P(wset), P(umask), P(prefix), P(counts), None, None, 0, P(ws),
                                             seq, None, B, ctypes.byref(sl), stream())
            else:
                rc = lib.omr_sum_list_build(P(masks_all), m, mstride, L.n, B, L.num_lanes, L.num_threads,
                                            ctypes.byref(sl), stream())
            assert rc == 0, lib.omr_last_error()
            out2 = out0.clone()
            rc = lib.omr_shard_sum_list_f32(P(own), P(recv), ctypes.byref(sl), m, L.n, B, L.num_lanes, L.num_threads,
                                            P(wset), P(prefix[m * (rows + 1):]), packed_out, P(out2), stream())
            assert rc == 0, lib.omr_last_error()
            torch.cuda.synchronize()
            outs.append(out2)
        assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32)), f"shard {s}: plan vs build list"
        o = outs[0].cpu().numpy()
        if packed_out:
            blocks = [r * L.num_lanes + ln for r in range(r0, r1) for ln in range(L.num_lanes)
                      if (int(ws_np[r]) >> ln) & 1]
            exp = np.concatenate([full[b * B:(b + 1) * B] for b in blocks]) if blocks else np.zeros(0, np.float32)
            assert (o[:exp.size].view(np.uint32) == exp.view(np.uint32)).all(), f"shard {s} packed"
        else:
            exp = (bufs[me].copy() if colocated else np.zeros(L.n, np.float32))
            wsb = np.repeat(np.array([(int(ws_np[r]) >> ln) & 1 for r in range(rows) for ln in range(L.num_lanes)],
                                     dtype=bool), B)
            mine = np.zeros(L.n, dtype=bool)
            mine[r0 * rowf:r1 * rowf] = True
            exp[mine & wsb] = full[mine & wsb]
            assert (o.view(np.uint32) == exp.view(np.uint32)).all(), f"shard {s} dense"
