#!/usr/bin/env python3
"""Where the round-3 shard sum's time goes, at config 4's 8-worker shard (tools/tune/shard_r03.hip, a stamped copy of
the product kernel): batch-timed windows of 16 / 32 / 64 pair slots, grids, and a per-wave timeline of the phases
(index data consumed, pair list written, first window summed, end with its stores acknowledged).  Outputs are
checked bit for bit against the product (round 3's omr_shard_sum_cols_f32, now tools/tune/plan_r04.hip).
usage: python tools/tune_shard_r03.py [--rounds 8] [--reps 20]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tune_round_r03 as r03  # noqa: E402
from omr import _lib  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "shard_r03.hip")
LIB = os.path.join(ROOT, "build", "libtune_shard_r03.so")


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_shard.argtypes = [i, i, vp, u32, vp, vp, vp, u32, u64, u64, vp, vp, u64, u64, u64, u32, u32, u32, vp, vp,
                               ctypes.c_uint, vp]
    lib.tune_shard_units.restype = ctypes.c_uint
    lib.tune_shard_units.argtypes = [u64, u64, u32, u32, u32, i]
    return lib


def main():
    ap = r03.parser()
    a = ap.parse_args()
    torch.cuda.init()
    tl = load()
    lib = _lib.load()
    tcols = r03.load_r04()  # (round 3's column-stream sum left the product in round 5: tools/tune/plan_r04.hip)
    D = r03.setup(a)
    L, m, rows, B, NB = D["L"], D["m"], D["rows"], D["B"], D["NB"]
    st, dev = D["st"], D["dev"]
    r0, r1 = D["r0"], D["r1"]
    roff = D["roff"].ctypes.data_as(ctypes.c_void_p)
    x0 = D["xs"][0]
    ref = x0.clone()
    assert tcols.tune_shard_sum_cols_r04(x0.data_ptr(), 0, D["recv_c"].data_ptr(), roff, D["masks_all"].data_ptr(), m,
                                      D["mstride"], 2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), L.n, B, NB,
                                      L.num_threads, r0, r1, 0, ref.data_ptr(), st) == 0
    units = tl.tune_shard_units(r0, r1, NB, D["S"], D["gps"], 1)
    nw = max(units, 2048 * 4)
    tlb = torch.zeros(nw * 8, dtype=torch.int64, device=dev)

    def run(v, stamp, out, grid=0):
        return tl.tune_shard(v, stamp, x0.data_ptr(), 0, D["recv_c"].data_ptr(), roff, D["masks_all"].data_ptr(), m,
                             D["mstride"], 2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), rows, r0, r1, NB,
                             D["S"], D["gps"], out.data_ptr(), tlb.data_ptr(), grid, st)

    cases = [(v, g) for v in (0, 1, 2) for g in (0, 128, 64)]
    names = {0: "window 32 (product)", 1: "window 16", 2: "window 64"}
    for v, g in cases:
        o = x0.clone()
        assert run(v, 0, o, g) == 0
        torch.cuda.synchronize()
        assert torch.equal(o.view(torch.int32), ref.view(torch.int32)), (v, g)
    outs = [x0.clone() for _ in range(2)]
    times = {c: [] for c in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for c in cases:
            e0.record()
            for i in range(a.reps):
                run(c[0], 0, outs[i % 2], c[1])
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[c].append(e0.elapsed_time(e1) / a.reps)
    sbytes = 45898752
    print(f"## shard 0 of {m}, {units} units: {sbytes} algorithmic bytes", flush=True)
    for c in sorted(cases, key=lambda c: np.median(times[c])):
        t = np.median(times[c]) * 1e-3
        print(f"{names[c[0]]:22s} grid {c[1] or 'auto':>5}  median {t * 1e6:7.2f} us  {sbytes / t / 1e9:7.1f} GB/s",
              flush=True)
    # per-wave timeline of the product's window (s_memrealtime ticks at 100 MHz)
    for v in (0,):
        tlb.zero_()
        run(v, 1, outs[0])
        torch.cuda.synchronize()
        t = tlb.view(-1, 8)[:units // 1].cpu().numpy().astype(np.int64)
        t = t[t[:, 0] > 0]
        base = t[:, 0].min()
        print(f"## timeline ({names[v]}, {len(t)} waves; us from the first wave's start)", flush=True)
        for col, what in ((0, "start"), (1, "index consumed"), (2, "pairs written"), (3, "first window summed"),
                          (4, "end, stores acked")):
            vals = (t[t[:, col] > 0, col] - base) / 100.0
            if vals.size == 0:
                continue
            print(f"  {what:22s} p10 {np.percentile(vals, 10):7.2f}  p50 {np.percentile(vals, 50):7.2f}  "
                  f"p90 {np.percentile(vals, 90):7.2f}  max {vals.max():7.2f}", flush=True)
        print(f"  units per wave: {np.bincount(t[:, 5].astype(np.int64)).tolist()}", flush=True)


if __name__ == "__main__":
    main()
