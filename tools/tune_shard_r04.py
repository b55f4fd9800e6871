#!/usr/bin/env python3
"""Round 4: the shard sum at config 4's 8-worker shard (tools/tune_round_r03.py's setup: 8 x 256 MiB, -r 0.095,
shard 0 of 8, column-ordered streams from the fused pack), the round-3 kernel (tools/tune/shard_r03.hip's copy)
against the product's (omr_shard_sum_cols_f32), batch-timed with events, interleaved, outputs checked bit for bit.
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


def main():
    ap = r03.parser()
    ap.add_argument("--rotate", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.init()
    tl = s03.load()
    lib = _lib.load()
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
        return lib.omr_shard_sum_cols_f32(x.data_ptr(), 0, rc.data_ptr(), roff, D["masks_all"].data_ptr(), m,
                                          D["mstride"], 2 * rows, D["prefix"].data_ptr(), D["wset"].data_ptr(), L.n, B,
                                          NB, L.num_threads, r0, r1, 0, out.data_ptr(), st)

    cases = {"round-3 kernel (copy)": r03k, "product (round 4)": prod}
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


if __name__ == "__main__":
    main()
