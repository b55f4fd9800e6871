#!/usr/bin/env python3
"""Round 4: the shard sum at config 4's 8-worker shard (tools/tune_round_r03.py's setup: 8 x 256 MiB, -r 0.095,
shard 0 of 8, column-ordered streams from the fused pack), the round-3 kernel (tools/tune/shard_r03.hip's copy)
against the product's (round 3's omr_shard_sum_cols_f32, now tools/tune/plan_r04.hip), batch-timed with events, interleaved, outputs checked bit for bit.
Four rotating output buffers and --rotate input sets (separate worker tensors / receive streams), so a launch does not
find the previous launch's data in the 256 MiB Infinity Cache.
usage: python tools/tune_shard_r04.py [--rounds 8] [--reps 20]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tune_round_r03 as r03  # noqa: E402
import tune_shard_r03 as s03  # noqa: E402
from omr import _lib  # noqa: E402


SRC4 = os.path.join(ROOT, "tools", "tune", "shard_r04.hip")
POLICIES = ("plain", "nt", "sc0 sc1")
LIB4 = os.path.join(ROOT, "build", "libtune_shard_r04.so")


def load4():
    """The stamped copy of the product kernel (tools/make_shard_r04.py writes its source)."""
    if not os.path.exists(LIB4) or os.path.getmtime(LIB4) < os.path.getmtime(SRC4):
        os.makedirs(os.path.dirname(LIB4), exist_ok=True)
        import subprocess
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB4, SRC4], check=True)
    lib = ctypes.CDLL(LIB4)
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    lib.tune_shard4.argtypes = [vp, u32, vp, vp, vp, u32, u64, u64, vp, vp, u64, u64, u64, u32, u32, u32, vp, vp, vp,
                                ctypes.c_int]
    lib.tune_shard4_list.argtypes = [vp, vp, vp, vp, u64, u32, u64, u32, vp, vp, vp]
    return lib


def timeline(tl, units, what, detail=False):
    t = tl.view(-1, 8)[:units].cpu().numpy().astype(np.int64)
    t = t[t[:, 0] > 0]
    base = t[:, 0].min()
    if detail:  # the end time by XCD and by the unit's pair count
        end = (t[:, 4] - base) / 100.0
        for x in sorted(set(t[:, 6].tolist())):
            sel = t[:, 6] == x
            print(f"  XCC {x}: {sel.sum():4d} waves, end p50 {np.median(end[sel]):6.2f} max {end[sel].max():6.2f}",
                  flush=True)
        for lo, hi in ((0, 16), (16, 24), (24, 32), (32, 48), (48, 64), (64, 999)):
            sel = (t[:, 7] >= lo) & (t[:, 7] < hi)
            if sel.any():
                print(f"  pairs [{lo:3d},{hi:3d}): {sel.sum():4d} waves, end p50 {np.median(end[sel]):6.2f} "
                      f"max {end[sel].max():6.2f}", flush=True)
    print(f"## timeline ({what}, {len(t)} waves; us from the first wave's entry)", flush=True)
    for col, name in ((0, "entry"), (1, "index consumed"), (2, "pairs written"), (3, "first window summed"),
                      (4, "end, stores acked")):
        vals = (t[t[:, col] > 0, col] - base) / 100.0
        if vals.size:
            print(f"  {name:22s} p10 {np.percentile(vals, 10):7.2f}  p50 {np.percentile(vals, 50):7.2f}  "
                  f"p90 {np.percentile(vals, 90):7.2f}  max {vals.max():7.2f}", flush=True)


def main():
    ap = r03.parser()
    ap.add_argument("--rotate", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.init()
    tl = s03.load()
    lib = _lib.load()
    tcols = r03.load_r04()  # (round 3's column-stream sum left the product in round 5: tools/tune/plan_r04.hip)
    D = r03.setup(a)
    L, m, rows, B, NB = D["L"], D["m"], D["rows"], D["B"], D["NB"]
    st = D["st"]
    r0, r1 = D["r0"], D["r1"]
    roff = D["roff"].ctypes.data_as(ctypes.c_void_p)
    # input sets: the same streams and own tensor, copied (the sums are identical; the bytes live elsewhere in HBM)
    sets = [(D["xs"][0], D["recv_c"])]
    for _ in range(a.rotate - 1):
        sets.append((D["xs"][0].clone(), D["recv_c"].clone()))
    outs = [D["xs"][0].clone() for _ in range(4)]
    units = tl.tune_shard_units(r0, r1, NB, D["S"], D["gps"], 1)
    tlb = torch.zeros(max(units, 8192) * 8, dtype=torch.int64, device=D["dev"])

    def r03k(k, out):
        x, rc = sets[k % len(sets)]
        return tl.tune_shard(0, 0, x.data_ptr(), 0, rc.data_ptr(), roff, D["masks_all"].data_ptr(), m, D["mstride"],
                             2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), rows, r0, r1, NB, D["S"],
                             D["gps"], out.data_ptr(), tlb.data_ptr(), 0, st)

    def prod(k, out):
        x, rc = sets[k % len(sets)]
        return tcols.tune_shard_sum_cols_r04(x.data_ptr(), 0, rc.data_ptr(), roff, D["masks_all"].data_ptr(), m,
                                          D["mstride"], 2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), L.n, B,
                                          NB, L.num_threads, r0, r1, 0, out.data_ptr(), st)

    # the pair list of shard 0, built once (the round builds it in its plan launch: omr_round_plan_list)
    units_l, cap = ctypes.c_uint64(), ctypes.c_uint32()
    _lib.check(lib.omr_sum_list_geometry(L.n, B, NB, L.num_threads, r0, r1, m, ctypes.byref(units_l),
                                         ctypes.byref(cap)), "geometry")
    lrec = torch.empty(units_l.value * cap.value, dtype=torch.int64, device=D["dev"])
    lcnt = torch.empty(units_l.value, dtype=torch.int32, device=D["dev"])
    sls = []
    for k in range(len(sets)):  # (one list per input set: the same pairs, different receive buffers)
        sl = _lib.SumList(lrec.data_ptr(), lcnt.data_ptr(), r0, r1, 2 * rows, 0)
        for w in range(m):
            sl.recv_offsets[w] = int(D["roff"][w])
        sls.append(sl)
    _lib.check(lib.omr_sum_list_build(D["masks_all"].data_ptr(), m, D["mstride"], L.n, B, NB, L.num_threads,
                                      ctypes.byref(sls[0]), st), "omr_sum_list_build")

    def plist(k, out):
        x, rc = sets[k % len(sets)]
        return lib.omr_shard_sum_list_f32(x.data_ptr(), rc.data_ptr(), ctypes.byref(sls[k % len(sets)]), m, L.n, B,
                                          NB, L.num_threads, D["wset"].data_ptr(),
                                          D["prefix"][m * (rows + 1):].data_ptr(), 0, out.data_ptr(), st)

    t4 = load4()

    def stamped(policy, ur=32):
        def f(k, out):
            x, rc = sets[k % len(sets)]
            return t4.tune_shard4(x.data_ptr(), 0, rc.data_ptr(), roff, D["masks_all"].data_ptr(), m, D["mstride"],
                                  2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), rows, r0, r1, NB, D["S"],
                                  D["gps"], out.data_ptr(), tlb.data_ptr(), st, policy, ur)
        return f

    cases = {"round-3 kernel (copy)": r03k, "product (round 4)": prod, "product, pair list (round 4)": plist}
    for pol, pname in enumerate(POLICIES):
        cases[f"stamped copy, {pname} stores"] = stamped(pol)
    cases["stamped copy, sc0 sc1 stores, 16-row units"] = stamped(2, 16)
    ref = D["xs"][0].clone()
    assert r03k(0, ref) == 0
    for name, f in cases.items():
        for k in range(len(sets)):
            o = D["xs"][0].clone()
            assert f(k, o) == 0, name
            torch.cuda.synchronize()
            assert torch.equal(o.view(torch.int32), ref.view(torch.int32)), (name, k)
    times = {c: [] for c in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for name, f in cases.items():
            e0.record()
            for i in range(a.reps):
                f(i, outs[i % 4])
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) / a.reps)
    sbytes = 45898752
    print(f"## shard 0 of {m}, {units} units, {len(sets)} input sets: {sbytes} algorithmic bytes", flush=True)
    for name in sorted(cases, key=lambda c: np.median(times[c])):
        t = np.median(times[name]) * 1e-3
        print(f"{name:26s} median {t * 1e6:7.2f} us  {sbytes / t / 1e9:7.1f} GB/s  "
              f"(min {min(times[name]) * 1e3:.2f} max {max(times[name]) * 1e3:.2f} us)", flush=True)
    for pol, ur in ((0, 32), (2, 32), (2, 16)):  # the product kernel's phases (stamped copy), a cold and a warm launch
        for k in range(2):
            tlb.zero_()
            stamped(pol, ur)(k, outs[0])
            torch.cuda.synchronize()
            timeline(tlb, units * 32 // ur, f"product kernel, stamped copy, {POLICIES[pol]} stores, {ur}-row units, "
                     f"launch {k}", detail=k == 1)
    for k in range(2):  # the pair-list kernel's phases (index consumed = its records loaded)
        tlb.zero_()
        x, rc = sets[k % len(sets)]
        t4.tune_shard4_list(x.data_ptr(), rc.data_ptr(), lrec.data_ptr(), lcnt.data_ptr(), units_l.value, cap.value,
                            r0, NB, outs[0].data_ptr(), tlb.data_ptr(), st)
        torch.cuda.synchronize()
        timeline(tlb, units, f"pair-list kernel, stamped copy, launch {k}")


if __name__ == "__main__":
    main()
