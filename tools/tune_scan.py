#!/usr/bin/env python3
"""Time k_scan1 shape variants and HBM calibration kernels side by side (one process, interleaved rounds).

usage: python tools/tune_scan.py [--size-mib 256] [--rounds 20] [--reps 5]
Builds omnireduce-rdma-demo_amd/tools/tune/scan_variants.hip into build/libtune.so (hipcc, gfx950)."""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, ops  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "scan_variants.hip")
LIB = os.path.join(ROOT, "build", "libtune.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_scan.argtypes = [i, vp, vp, vp, vp, u64, u32, u32, ctypes.c_uint, vp]
    lib.tune_read.argtypes = [i, i, vp, u64, vp, ctypes.c_uint, vp]
    lib.tune_copy.argtypes = [i, vp, vp, u64, ctypes.c_uint, vp]
    lib.tune_variant_name.restype = ctypes.c_char_p
    return lib


VARIANTS = list(range(31))
CAPS = (1024, 2048, 4096)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default="")
    ap.add_argument("--variants", default="")
    ap.add_argument("--caps", default="")
    ap.add_argument("--step", action="store_true",
                    help="time [variant scan + product k_next] steps with events only around each batch")
    ap.add_argument("--no-calib", action="store_true")
    ap.add_argument("--inplace", action="store_true", help="out aliases x (the reference's in-place result)")
    args = ap.parse_args()
    global VARIANTS, CAPS
    if args.variants:
        VARIANTS = [int(v) for v in args.variants.split(",")]
    if args.caps:
        CAPS = tuple(int(v) for v in args.caps.split(","))
    torch.cuda.init()
    lib = build()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(args.size_mib << 20, args.block_size)
    bm = ops.gen_bitmap(0, args.density, L.nb)
    bmt = torch.from_numpy(bm).to(dev)
    NSET = 4
    xs = [ops.fill_blocks(bmt, L) for _ in range(NSET)]
    outs_sep = [torch.zeros(L.n, device=dev) for _ in range(NSET)]
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    masks = torch.zeros(L.rows, dtype=torch.int64, device=dev)
    sink = torch.zeros(1 << 20, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    heads = ((np.arange(L.nb) // L.num_lanes) % L.rows_per_part) == 0
    kbytes = L.nbytes + int(np.count_nonzero(bm.astype(bool) | heads)) * L.block_size * 4 + L.nb * 4 + L.rows * 8

    cases = []
    for v in VARIANTS:
        for cap in CAPS:
            for mode in (("sep", "inpl") if args.inplace else ("sep",)):
                outs = xs if mode == "inpl" else outs_sep
                name = lib.tune_variant_name(v).decode()
                cases.append((f"{name} cap{cap} {mode}", kbytes,
                              lambda k, v=v, cap=cap, outs=outs: lib.tune_scan(
                                  v, xs[k].data_ptr(), outs[k].data_ptr(), flags.data_ptr(), masks.data_ptr(),
                                  L.rows, L.num_lanes, L.rows_per_part, cap, st)))
    next_out = torch.empty(L.nb, dtype=torch.int32, device=dev)
    if args.step:
        lib_omr = __import__("omr")._lib.load()
        base_cases = cases
        cases = []
        for name, nb_, fn in base_cases:
            def stepfn(k, fn=fn):
                rc = fn(k)
                lib_omr.omr_next_offsets(masks.data_ptr(), 1, L.n, L.block_size, L.num_lanes, L.num_threads,
                                         next_out.data_ptr(), st)
                return rc
            cases.append((name + " +next", nb_, stepfn))
    for nt in ((0, 1) if not args.no_calib else ()):
        for loads in (16, 32):
            for g in (1024, 2048, 4096):
                cases.append((f"read nt{nt} L{loads} g{g}", L.nbytes,
                              lambda k, nt=nt, loads=loads, g=g: lib.tune_read(nt, loads, xs[k].data_ptr(), L.n,
                                                                               sink.data_ptr(), g, st)))
        for g in (2048, 8192, 32768):
            cases.append((f"copy nt{nt} g{g}", 2 * L.nbytes,
                          lambda k, nt=nt, g=g: lib.tune_copy(nt, xs[k].data_ptr(), outs_sep[k].data_ptr(), L.n, g,
                                                              st)))
    # correctness of every scan variant against the product kernel
    ref = ops.scan(xs[0], L)
    for ci, (name, _, fn) in enumerate(cases):
        if not name.startswith(("read", "copy", "col")) and "nostore" not in name:
            flags.zero_(); masks.zero_()
            assert fn(0) == 0
            torch.cuda.synchronize()
            assert torch.equal(flags, ref.flags[0]) and torch.equal(masks, ref.masks[0]), name
    times = {name: [] for name, _, _ in cases}
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
    k = 0
    for r in range(args.rounds):
        for name, _, fn in cases:
            for e0, e1 in ev:
                e0.record()
                fn(k % NSET)
                e1.record()
                k += 1
            torch.cuda.synchronize()
            if r > 0:
                times[name] += [a.elapsed_time(b) for a, b in ev]
    res = []
    for name, nbytes, _ in cases:
        t = np.array(times[name]) * 1e-3
        res.append({"case": name, "median_us": float(np.median(t) * 1e6), "min_us": float(t.min() * 1e6),
                    "GBps_median": nbytes / np.median(t) / 1e9, "GBps_best": nbytes / t.min() / 1e9})
    for r_ in sorted(res, key=lambda d: d["median_us"] if not d["case"].startswith(("read", "copy")) else 1e9):
        print(f"{r_['case']:32s} median {r_['median_us']:8.2f} us  min {r_['min_us']:8.2f} us  "
              f"{r_['GBps_median']:8.1f} GB/s (best {r_['GBps_best']:8.1f})")
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"size_mib": args.size_mib, "kernel_bytes": kbytes, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
