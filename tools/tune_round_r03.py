#!/usr/bin/env python3
"""Rounds 3-5: the multi-rank round's worker and aggregator kernels at config-4 shapes on one MI355X (8 workers x 256 MiB,
-r 0.095, seeds 1..8; rank 0's view: worker 0 and aggregator of shard 0 of 8).  Forms that lost (round 4's row-chunk
plan, round 3's column-stream shard sum, the round-3/4 plan) come from tools/tune/plan_r04.hip (built on first use).

Worker side, per launch (algorithmic bytes in brackets):
  scan       omr_worker_scan_f32             [S + nb*8 + rows*8]
  scan+pack  omr_worker_scan_pack_f32        [+ the other shards' non-zero blocks written + table]   (the product)
  pack       omr_move_blocks_f32 (round 2's separate pack pass)  [its blocks read + written]
Aggregator side, shard 0's sums from 8 contributions (own in place + 7 received streams) [received + own + write-set
blocks, as tools/tune_round_r02.py counts them]:
  round-2 k_shard_sum (tools/tune/round_r02.hip), the product's k_shard_sum over row-ordered streams
  (omr_shard_sum_f32) and over the fused pack's column-ordered streams (round 3's omr_shard_sum_cols_f32, from
  tools/tune/plan_r04.hip since round 5).
Every variant's output is checked bit for bit against the others.  Batch-timed with events, interleaved.
usage: python tools/tune_round_r03.py [--rounds 10] [--reps 20]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, _lib, ops  # noqa: E402
import tune_round_r02 as r02  # noqa: E402


def popc(a):
    return int(sum(bin(int(v) & 0xFFFFFFFFFFFFFFFF).count("1") for v in a))


def parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--only", default="", help="time only the cases whose name contains this (PMC passes)")
    ap.add_argument("--json", default="", help="also write {case: {us, bytes}} here")
    ap.add_argument("--check-slots", type=int, default=-1,
                    help="the round check case reads this many slots per worker (default: the round's count)")
    return ap


def setup(a):
    """Config-4 shapes on one device: m workers' scans with the fused pack, the plan over the all-gathered arrays, and
    shard 0's received streams in both layouts (column-ordered from the fused pack, row-ordered from k_move)."""
    lib = _lib.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    L = Layout.from_bytes(256 << 20, 256)
    m = naggs = a.workers
    rows, B, NB = L.rows, 256, L.num_lanes
    S_, gps, ent = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    assert lib.omr_pack_geometry(L.n, B, NB, L.num_threads, ctypes.byref(S_), ctypes.byref(gps), ctypes.byref(ent)) == 0
    ent = ent.value
    mstride = rows + (ent + 1) // 2
    bounds = np.array([s * rows // naggs for s in range(naggs + 1)], dtype=np.uint64)
    bptr = bounds.ctypes.data_as(ctypes.c_void_p)
    xs = [ops.fill_blocks(torch.from_numpy(ops.gen_bitmap(w, a.density, L.nb)).to(dev), L) for w in range(m)]
    wsb = lib.omr_scan_workspace_bytes(L.n, B, NB, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    flags = torch.empty(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.empty(L.nb, dtype=torch.int32, device=dev)
    # every worker's scan + fused pack into its slot of the all-gathered array, and its send buffer
    masks_all = torch.zeros(m * mstride, dtype=torch.int64, device=dev)
    sends, cnts = [], []
    for w in range(m):
        slot = masks_all[w * mstride:(w + 1) * mstride]
        send = torch.empty(L.n, dtype=torch.float32, device=dev)
        cnt = torch.zeros(naggs, dtype=torch.int32, device=dev)
        _lib.check(lib.omr_worker_scan_pack_f32(xs[w].data_ptr(), L.n, B, NB, L.num_threads, flags.data_ptr(),
                                                nxt.data_ptr(), slot.data_ptr(), None, bptr, naggs, w, send.data_ptr(),
                                                cnt.data_ptr(), slot[rows:].data_ptr(), ws.data_ptr(), wsb, st),
                   "omr_worker_scan_pack_f32")
        sends.append(send)
        cnts.append(cnt)
    torch.cuda.synchronize()
    cnts = [c.cpu().numpy() for c in cnts]
    wset = torch.empty(rows, dtype=torch.int64, device=dev)
    umask = torch.empty(rows, dtype=torch.int64, device=dev)
    prefix = torch.empty((m + 1) * (rows + 1), dtype=torch.int32, device=dev)
    counts = torch.empty((m + 1) * (naggs + 1), dtype=torch.int64, device=dev)
    bdev = torch.from_numpy(bounds.astype(np.int64)).to(dev)
    pws5 = torch.zeros(int(lib.omr_round_plan_workspace_words()), dtype=torch.int64, device=dev)
    _lib.check(lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                       naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                       counts.data_ptr(), None, None, 0, pws5.data_ptr(), 1, None, B, None, st), "plan")
    # the round-2 layout: masks [m][rows] contiguous, row-ordered streams packed by k_move
    masks = torch.stack([masks_all[w * mstride:w * mstride + rows] for w in range(m)]).contiguous()
    torch.cuda.synchronize()
    r0, r1 = int(bounds[0]), int(bounds[1])
    pre = prefix.view(m + 1, rows + 1)
    per = [cnts[w][0] for w in range(m)]
    roff = np.zeros(m, dtype=np.uint64)
    acc = 0
    for w in range(1, m):
        roff[w] = acc
        acc += int(per[w])
    recv_c = torch.empty(max(acc, 1) * B, dtype=torch.float32, device=dev)  # column-ordered (fused pack) streams
    recv_r = torch.empty(max(acc, 1) * B, dtype=torch.float32, device=dev)  # row-ordered (k_move) streams
    for w in range(1, m):
        k0, k = int(roff[w]), int(per[w])
        recv_c[k0 * B:(k0 + k) * B].copy_(sends[w][r0 * NB * B:(r0 * NB + k) * B])
        _lib.check(lib.omr_move_blocks_f32(xs[w].data_ptr(), recv_r[k0 * B:].data_ptr(), 0, masks[w].data_ptr(),
                                           pre[w].data_ptr(), rows, NB, B, r1, rows, st), "pack")
    torch.cuda.synchronize()
    return dict(L=L, m=m, naggs=naggs, rows=rows, B=B, NB=NB, ent=ent, mstride=mstride, bounds=bounds, bptr=bptr,
                xs=xs, wsb=wsb, ws=ws, flags=flags, nxt=nxt, masks_all=masks_all, sends=sends, cnts=cnts, wset=wset,
                umask=umask, prefix=prefix, counts=counts, bdev=bdev, masks=masks, r0=r0, r1=r1, pre=pre, roff=roff,
                acc=acc, recv_c=recv_c, recv_r=recv_r, pws5=pws5, S=S_.value, gps=gps.value, dev=dev, st=st)


TUNE_SRC = os.path.join(ROOT, "tools", "tune", "plan_r04.hip")
TUNE_LIB = os.path.join(ROOT, "gpurun_out", "tune", "libplan_r04.so")


def load_r04():
    """tools/tune/plan_r04.hip (the losing forms, kept for A/B), compiled on first use."""
    import subprocess
    if not os.path.exists(TUNE_LIB) or os.path.getmtime(TUNE_LIB) < os.path.getmtime(TUNE_SRC):
        os.makedirs(os.path.dirname(TUNE_LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", TUNE_LIB, TUNE_SRC], check=True)
    t = ctypes.CDLL(TUNE_LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    plan_args = [vp, u32, u64, u64, u32, u32, vp, u32, vp, vp, vp, vp, vp, vp, u32, vp, vp, u32, vp, u32, vp, vp]
    t.tune_round_plan_list_r04.argtypes = plan_args
    t.tune_round_plan_ws_r04.argtypes = plan_args
    t.tune_round_plan_workspace_words_r04.restype = u64
    t.tune_shard_sum_cols_r04.argtypes = [vp, u32, vp, vp, vp, u32, u64, u64, vp, vp, u64, u32, u32, u32, u64, u64, i,
                                          vp, vp]
    return t


def main():
    a = parser().parse_args()
    torch.cuda.init()
    tl = r02.load()
    t4 = load_r04()
    lib = _lib.load()
    print("# setting up config 4's shapes", flush=True)
    D = setup(a)
    print("# set up", flush=True)
    L, m, naggs, rows, B, NB, ent, mstride = (D[k] for k in ("L", "m", "naggs", "rows", "B", "NB", "ent", "mstride"))
    bounds, bptr, xs, wsb, ws, flags, nxt = (D[k] for k in ("bounds", "bptr", "xs", "wsb", "ws", "flags", "nxt"))
    masks_all, wset, umask, prefix, counts, bdev = (D[k] for k in ("masks_all", "wset", "umask", "prefix", "counts",
                                                                     "bdev"))
    masks, r0, r1, pre, roff, acc, recv_c, recv_r = (D[k] for k in ("masks", "r0", "r1", "pre", "roff", "acc",
                                                                   "recv_c", "recv_r"))
    dev, st = D["dev"], D["st"]
    roff_c = roff.ctypes.data_as(ctypes.c_void_p)
    roff_t = (ctypes.c_uint64 * m)(*[int(v) for v in roff])

    def sum_r02(out):
        return tl.tune_shard_sum(0, xs[0].data_ptr(), 0, recv_r.data_ptr(), roff_t, masks.data_ptr(), m,
                                 prefix.data_ptr(), wset.data_ptr(), rows, r0, r1, NB, 0, out.data_ptr(), 0, st)

    def sum_rows(out):
        return lib.omr_shard_sum_f32(xs[0].data_ptr(), 0, recv_r.data_ptr(), roff_c, masks.data_ptr(), m,
                                     prefix.data_ptr(), wset.data_ptr(), rows, r0, r1, NB, B, 0, out.data_ptr(), st)

    def sum_cols(out):  # round 3's column-stream sum (tools/tune/plan_r04.hip)
        return t4.tune_shard_sum_cols_r04(xs[0].data_ptr(), 0, recv_c.data_ptr(), roff_c, masks_all.data_ptr(), m,
                                          mstride, 2 * rows, prefix.data_ptr(), wset.data_ptr(), L.n, B, NB,
                                          L.num_threads, r0, r1, 0, out.data_ptr(), st)

    # the pair list of shard 0 (built once here; the round builds it in its plan launch, timed below)
    units, cap = ctypes.c_uint64(), ctypes.c_uint32()
    _lib.check(lib.omr_sum_list_geometry(L.n, B, NB, L.num_threads, r0, r1, m, ctypes.byref(units), ctypes.byref(cap)),
               "geometry")
    lrec = torch.empty(units.value * cap.value, dtype=torch.int64, device=dev)
    lcnt = torch.empty(units.value, dtype=torch.int32, device=dev)
    sl = _lib.SumList(lrec.data_ptr(), lcnt.data_ptr(), r0, r1, 2 * rows, 0)
    for w in range(m):
        sl.recv_offsets[w] = int(roff[w])
    _lib.check(lib.omr_sum_list_build(masks_all.data_ptr(), m, mstride, L.n, B, NB, L.num_threads, ctypes.byref(sl),
                                      st), "omr_sum_list_build")
    torch.cuda.synchronize()
    print("# pair list built", flush=True)

    def sum_list(out):
        return lib.omr_shard_sum_list_f32(xs[0].data_ptr(), recv_c.data_ptr(), ctypes.byref(sl), m, L.n, B, NB,
                                          L.num_threads, wset.data_ptr(), prefix[m * (rows + 1):].data_ptr(), 0,
                                          out.data_ptr(), st)

    def env_case(fn, var, val):
        def run(out):
            os.environ[var] = val
            try:
                return fn(out)
            finally:
                del os.environ[var]
        return run

    sums = {"round-2 k_shard_sum (rows)": sum_r02, "product k_shard_sum (rows)": sum_rows,
            "round-3 k_shard_sum (cols)": sum_cols, "product k_shard_sum_list (pairs from the plan)": sum_list}
    ref = None
    for name, fn in sums.items():
        o = xs[0].clone()
        print(f"# checking {name}", flush=True)
        assert fn(o) == 0, name
        torch.cuda.synchronize()
        print(f"# {name} ran", flush=True)
        if ref is None:
            ref = o
        assert torch.equal(o.view(torch.int32), ref.view(torch.int32)), f"{name} differs"
    # worker side: worker 0's scan alone, scan + fused pack, and the separate pack pass
    own_masks = torch.zeros(mstride, dtype=torch.int64, device=dev)
    send0 = torch.empty(L.n, dtype=torch.float32, device=dev)
    cntbig = torch.zeros(a.reps * naggs, dtype=torch.int32, device=dev)  # one fresh counter set per launch
    packed = torch.empty(L.n, dtype=torch.float32, device=dev)

    def scan():
        return lib.omr_worker_scan_f32(xs[0].data_ptr(), L.n, B, NB, L.num_threads, flags.data_ptr(), nxt.data_ptr(),
                                       own_masks.data_ptr(), None, ws.data_ptr(), wsb, st)

    def scan_pack(i=0):
        return lib.omr_worker_scan_pack_f32(xs[0].data_ptr(), L.n, B, NB, L.num_threads, flags.data_ptr(),
                                            nxt.data_ptr(), own_masks.data_ptr(), None, bptr, naggs, 0,
                                            send0.data_ptr(), cntbig[i * naggs:].data_ptr(),
                                            own_masks[rows:].data_ptr(), ws.data_ptr(), wsb, st)

    ns = int(lib.omr_round_check_slots(L.n, B, NB, L.num_threads))
    chk_slots = torch.zeros(ns, dtype=torch.int64, device=dev)
    done = torch.zeros(2, dtype=torch.int32, device=dev)  # (the scan's completion word, as the round passes it)

    def scan_pack_chk(i=0):  # the round's worker scan since round 6: + its round-check slots
        return lib.omr_worker_scan_pack_check_f32(xs[0].data_ptr(), L.n, B, NB, L.num_threads, flags.data_ptr(),
                                                  nxt.data_ptr(), own_masks.data_ptr(), None, bptr, naggs, 0,
                                                  send0.data_ptr(), cntbig[i * naggs:].data_ptr(),
                                                  own_masks[rows:].data_ptr(), ws.data_ptr(), wsb,
                                                  chk_slots.data_ptr(), 1, done.data_ptr(), st)

    def pack():
        return lib.omr_move_blocks_f32(xs[0].data_ptr(), packed.data_ptr(), 0, masks[0].data_ptr(), pre[0].data_ptr(),
                                       rows, NB, B, r0, r1, st)

    unext = torch.empty(L.nb, dtype=torch.int32, device=dev)

    # the round's own setting: tagged counts into pinned host memory (system-scope stores), the own masks and pack
    # counters cleared (scratch copies here), the pair list, no chain (bench asks for no union_next)
    pin = torch.zeros(4096, dtype=torch.int32).pin_memory()
    pin_d = ctypes.c_void_p()
    assert ctypes.CDLL("libamdhip64.so").hipHostGetDevicePointer(ctypes.byref(pin_d), ctypes.c_void_p(pin.data_ptr()),
                                                                 0) == 0
    cnt_d, flag_d = pin_d.value, pin_d.value + 4 * 2048  # (the notice: the round-3/4 form only)
    zmask = torch.empty(rows, dtype=torch.int64, device=dev)
    zcnt = torch.empty(naggs, dtype=torch.int32, device=dev)
    arrive = torch.zeros(1, dtype=torch.int32, device=dev)
    seqs = [1]
    pws5 = D["pws5"]

    def nseq():  # every product plan launch shares pws5: a fresh sequence number each
        seqs[0] += 1
        return seqs[0]

    def plan():  # the round's bookkeeping launch: write set, union, prefixes, counts, aggregator chain
        return lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                       naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                       counts.data_ptr(), None, None, 0, pws5.data_ptr(), nseq(), unext.data_ptr(), B,
                                       None, st)

    def plan_list():  # ... with shard 0's pair list built by the same launch (the round since round 3)
        return lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                       naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                       counts.data_ptr(), None, None, 0, pws5.data_ptr(), nseq(), unext.data_ptr(), B,
                                       ctypes.byref(sl), st)

    def plan_round():  # exactly the round's call (round 5's row-chunk plan)
        return lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                       naggs + 1, wset.data_ptr(), None, prefix.data_ptr(), cnt_d, zmask.data_ptr(),
                                       zcnt.data_ptr(), naggs, pws5.data_ptr(), nseq(), None, B, ctypes.byref(sl), st)

    chk_status = cnt_d + 12 * 1024  # (pinned, beside the counts and the round-3/4 notice)
    nchk = min(ns, mstride - rows) if a.check_slots < 0 else min(a.check_slots, mstride - rows)

    def plan_round_chk():  # the round's call since round 6: + the round check's workgroup (timing only: the words it
        # checks here are position-table entries, so its status reports a mismatch)
        return lib.omr_round_plan_check(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                        naggs + 1, wset.data_ptr(), None, prefix.data_ptr(), cnt_d, zmask.data_ptr(),
                                        zcnt.data_ptr(), naggs, pws5.data_ptr(), nseq(), None, B, ctypes.byref(sl),
                                        rows, nchk, chk_status, st)

    def plan_round_r04():  # the same call to the round-3/4 plan (one workgroup per mask array, arrival counter)
        seqs[0] += 1
        return t4.tune_round_plan_list_r04(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB,
                                           bdev.data_ptr(), naggs + 1, wset.data_ptr(), umask.data_ptr(),
                                           prefix.data_ptr(), cnt_d, zmask.data_ptr(), zcnt.data_ptr(), naggs,
                                           arrive.data_ptr(), flag_d, seqs[0], None, B, ctypes.byref(sl), st)

    pws = torch.zeros(t4.tune_round_plan_workspace_words_r04(), dtype=torch.int32, device=dev)

    def plan_ws():  # round 4's row-chunk form, the round's plan with the fused pack (tools/tune/plan_r04.hip)
        return t4.tune_round_plan_ws_r04(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                         naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                         counts.data_ptr(), None, None, 0, pws.data_ptr(), None, 0, unext.data_ptr(),
                                         B, None, st)

    def plan_nochain():  # the plan without the aggregator chain
        return lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                       naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                       counts.data_ptr(), None, None, 0, pws5.data_ptr(), nseq(), None, B, None, st)

    def plan_nochain_r04():  # the round-3/4 plan without the chain
        return t4.tune_round_plan_list_r04(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB,
                                           bdev.data_ptr(), naggs + 1, wset.data_ptr(), umask.data_ptr(),
                                           prefix.data_ptr(), counts.data_ptr(), None, None, 0, None, None, 0, None, B,
                                           None, st)

    def plan_ws_nochain():  # the row-chunk form without the chain
        return t4.tune_round_plan_ws_r04(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                                         naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(),
                                         counts.data_ptr(), None, None, 0, pws.data_ptr(), None, 0, None, B, None, st)

    def list_only():  # the pair list in a launch of its own
        return lib.omr_sum_list_build(masks_all.data_ptr(), m, mstride, L.n, B, NB, L.num_threads, ctypes.byref(sl),
                                      st)

    workers = {"scan (omr_worker_scan_f32)": scan, "scan + fused pack (product)": scan_pack,
               "scan + fused pack + round-check slots (the round's, round 6)": scan_pack_chk,
               "round plan as the round calls it + round check (round 6)": plan_round_chk,
               "pack pass (k_move, round 2)": pack, "round plan + chain (k_round_plan)": plan,
               "round plan + chain, row chunks (k_round_plan2)": plan_ws,
               "round plan, no chain (k_round_plan)": plan_nochain,
               "round plan, no chain (round-3/4 k_round_plan_r04)": plan_nochain_r04,
               "round plan, no chain, row chunks (k_round_plan2)": plan_ws_nochain,
               "round plan + chain + pair list": plan_list,
               "round plan as the round calls it (pair list, pinned counts)": plan_round,
               "round plan as the round calls it, round-3/4 form": plan_round_r04,
               "pair list alone (k_sum_list)": list_only}
    cases = {**sums, **workers}
    if a.only:
        cases = {k: v for k, v in cases.items() if a.only in k}
    outs = [xs[0].clone() for _ in range(2)]
    times = {k: [] for k in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print("# checked; timing", flush=True)
    for r in range(a.rounds):
        print(f"# round {r}", flush=True)
        for name, fn in cases.items():
            cntbig.zero_()
            e0.record()
            for i in range(a.reps):
                if name in sums:
                    fn(outs[i % 2])
                elif fn is scan_pack or fn is scan_pack_chk:
                    fn(i)
                else:
                    fn()
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) / a.reps)
    mk = masks.cpu().numpy().view(np.uint64)
    own_blocks = popc(mk[0][r0:r1])
    ub = popc(wset.cpu().numpy().view(np.uint64)[r0:r1])
    nc = int(acc)
    sbytes = (nc + own_blocks + ub) * B * 4
    other = popc(mk[0]) - own_blocks
    scan_b = L.nbytes + L.nb * 8 + rows * 8
    table_b = ent * 4 * (naggs - 1) // naggs
    wbytes = {"scan (omr_worker_scan_f32)": scan_b, "scan + fused pack (product)": scan_b + other * B * 4 + table_b,
              "pack pass (k_move, round 2)": 2 * other * B * 4,
              # reads every worker's masks; writes write set, union, m + 1 prefix arrays, counts, the union chain
              "round plan + chain (k_round_plan)": m * rows * 8 + 2 * rows * 8 + (m + 1) * (rows + 1) * 4 +
              L.nb * 4}
    # the pair list: reads every worker's mask rows of the shard and position-table entries, writes the records
    nrec = int(lcnt.sum().item())
    lbytes = m * (r1 - r0) * 8 + m * (ent // naggs) * 4 + nrec * 8 + units.value * 4
    wbytes["round plan + chain + pair list"] = wbytes["round plan + chain (k_round_plan)"] + lbytes
    wbytes["round plan + chain, row chunks (k_round_plan2)"] = wbytes["round plan + chain (k_round_plan)"]
    wbytes["round plan, no chain (k_round_plan)"] = wbytes["round plan + chain (k_round_plan)"] - L.nb * 4
    wbytes["round plan, no chain, row chunks (k_round_plan2)"] = wbytes["round plan, no chain (k_round_plan)"]
    wbytes["round plan, no chain (round-3/4 k_round_plan_r04)"] = wbytes["round plan, no chain (k_round_plan)"]
    # the round's call: no union stored, no chain; its own masks cleared (rows words), the pair list
    wbytes["round plan as the round calls it (pair list, pinned counts)"] = (
        m * rows * 8 + rows * 8 + (m + 1) * (rows + 1) * 4 + rows * 8 + lbytes)
    wbytes["round plan as the round calls it, round-3/4 form"] = (
        wbytes["round plan as the round calls it (pair list, pinned counts)"] + rows * 8)  # (+ its union)
    wbytes["pair list alone (k_sum_list)"] = lbytes
    # round 6: the scan's slots (8 B per workgroup) and the check's reads of every worker's slots
    wbytes["scan + fused pack + round-check slots (the round's, round 6)"] = (
        wbytes["scan + fused pack (product)"] + ns * 8)
    wbytes["round plan as the round calls it + round check (round 6)"] = (
        wbytes["round plan as the round calls it (pair list, pinned counts)"] + m * nchk * 8)
    report = {}
    print(f"## config 4 shapes, {m} workers, -r {a.density}: shard 0 write set {ub} blocks, received {nc}, own {own_blocks}: "
          f"{sbytes} B per shard sum; worker 0 packs {other} blocks", flush=True)
    for name in cases:
        t = np.median(times[name]) * 1e-3
        b = sbytes if name in sums else wbytes[name]
        report[name] = {"us": round(t * 1e6, 3), "algorithmic_bytes": int(b), "GBps": round(b / t / 1e9, 1)}
        print(f"{name:34s} median {t * 1e6:8.2f} us  {b:>11d} B  {b / t / 1e9:7.1f} GB/s  ({b / t / 8e12:.3f} of 8 TB/s)",
              flush=True)
    trio = ["scan (omr_worker_scan_f32)", "scan + fused pack (product)", "pack pass (k_move, round 2)"]
    if all(k in times and times[k] for k in trio):
        ts, tsp, tp = (np.median(times[k]) * 1e3 for k in trio)
        print(f"worker side per round: scan + pack pass {ts + tp:.2f} us -> fused {tsp:.2f} us", flush=True)
    if a.json:
        import json
        with open(a.json, "w") as f:
            json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
