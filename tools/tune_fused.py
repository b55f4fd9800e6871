#!/usr/bin/env python3
"""Time k_scan1f variants (waves per workgroup, loads in flight, XCD column mapping, segments per column K)
side by side in one process, interleaved rounds, in place as the bench runs (or --out-of-place); every variant is
checked against the product kernel's flags and next offsets first.  usage: python tools/tune_fused.py [--rounds 12]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, ops  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "fused_variants.hip")
LIB = os.path.join(ROOT, "build", "libtune_fused.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_fused.argtypes = [i, vp, vp, vp, vp, vp, u64, u32, u32, vp]
    lib.tune_fused_name.restype = ctypes.c_char_p
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=20, help="launches between one pair of events")
    ap.add_argument("--variants", default="", help="comma list of variant indices (default: all)")
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--out-of-place", action="store_true",
                    help="write each input set's sums into an output of its own (as the world-1 round does)")
    a = ap.parse_args()
    torch.cuda.init()
    if not os.path.exists(LIB):
        pass
    lib = build()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.size_mib << 20, a.block_size)
    bm = ops.gen_bitmap(0, a.density, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for _ in range(4)]
    outs = [x.clone() for x in xs] if a.out_of_place else xs
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    ref = ops.ScanSumPlan(L, 1, device=dev, fused=True).run([xs[0]], xs[0])
    torch.cuda.synchronize()
    heads = ((np.arange(L.nb) // L.num_lanes) % L.rows_per_part) == 0
    kbytes = L.nbytes + int(np.count_nonzero(bm.astype(bool) | heads)) * L.block_size * 4 + L.nb * 8
    cases = []
    # the product launch itself (its own shape choice), for reference
    pplan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
    plaunch = [pplan.bind(xs[k], outs[k], torch.cuda.current_stream()) for k in range(4)]
    cases.append(("product", lambda k: plaunch[k]() or 0))
    vids = [int(x) for x in a.variants.split(",")] if a.variants else list(range(lib.tune_fused_count()))
    for v in vids:
        for K in [int(x) for x in a.ks.split(",")]:
            name = f"{lib.tune_fused_name(v).decode()} K{K}"
            cases.append((name, lambda k, v=v, K=K: lib.tune_fused(v, xs[k].data_ptr(), outs[k].data_ptr(),
                                                                    flags.data_ptr(), nxt.data_ptr(), ws.data_ptr(),
                                                                    L.n, L.block_size, K, st)))
    for (name, fn), v in zip(cases[1:], [v for v in vids for _ in a.ks.split(",")]):
        flags.zero_(); nxt.zero_()
        assert fn(0) == 0, name
        torch.cuda.synchronize()
        if lib.tune_fused_checked(v):
            assert torch.equal(flags, ref.flags[0]) and torch.equal(nxt, ref.next_offsets[0]), name
    times = {n: [] for n, _ in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 0
    for r in range(a.rounds):  # per case: one event pair around a.reps back-to-back launches (bench.py's timing)
        for name, fn in cases:
            e0.record()
            for _ in range(a.reps):
                fn(k % 4)
                k += 1
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) / a.reps)
    for name, _ in sorted(cases, key=lambda c: np.median(times[c[0]])):
        t = np.array(times[name]) * 1e-3
        print(f"{name:22s} median {np.median(t)*1e6:8.2f} us  min {t.min()*1e6:8.2f} us  "
              f"{kbytes/np.median(t)/1e9:8.1f} GB/s")


if __name__ == "__main__":
    main()
