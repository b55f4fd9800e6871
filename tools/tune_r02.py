#!/usr/bin/env python3
"""Round-2 single-pass kernel study: time tools/tune/fused_r02.hip variants (decoupled stores k_scan1d vs the product
k_scan1f, ablations, the pure read of the same geometry) side by side in one process, interleaved rounds, in place as
bench.py runs.  Every full-output variant is first checked against the product kernel (flags, next offsets and the
out-of-place aggregated blocks, bit for bit).
usage: python tools/tune_r02.py [--size-mib 256 --block-size 256 --density 0.095 --ks 1]"""
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

SRC = os.path.join(ROOT, "tools", "tune", "fused_r02.hip")
LIB = os.path.join(ROOT, "build", "libtune_r02.so")


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_run.argtypes = [i, vp, vp, vp, vp, vp, u64, u32, u32, u32, vp]
    lib.tune_name.restype = ctypes.c_char_p
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=20, help="launches between one pair of events")
    ap.add_argument("--variants", default="", help="comma list of variant indices (default: all)")
    ap.add_argument("--ks", default="1")
    ap.add_argument("--occs", default="0", help="workgroups per CU forced with dynamic LDS (0 = natural)")
    a = ap.parse_args()
    torch.cuda.init()
    lib = load()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.size_mib << 20, a.block_size)
    bm = ops.gen_bitmap(0, a.density, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for _ in range(4)]
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    heads = ((np.arange(L.nb) // L.num_lanes) % L.rows_per_part) == 0
    kbytes = L.nbytes + int(np.count_nonzero(bm.astype(bool) | heads)) * L.block_size * 4 + L.nb * 8
    vids = [int(x) for x in a.variants.split(",")] if a.variants else list(range(lib.tune_count()))
    ks = [int(x) for x in a.ks.split(",")]
    cases = []
    occs = [int(x) for x in a.occs.split(",")]
    for v in vids:
        for K in ks:
            for o in (occs if v else [0]):
                cases.append((f"{lib.tune_name(v).decode()} K{K}" + (f" occ{o}" if o else ""), v, (K, o)))

    def run(v, Ko, x, out):
        return lib.tune_run(v, x.data_ptr(), out.data_ptr() if out is not None else None, flags.data_ptr(),
                            nxt.data_ptr(), ws.data_ptr(), L.n, L.block_size, Ko[0], Ko[1], st)

    ref_out = torch.zeros(L.n, device=dev)
    assert run(0, (ks[0], 0), xs[0], ref_out) == 0
    torch.cuda.synchronize()
    ref_flags, ref_next = flags.clone(), nxt.clone()
    for name, v, K in cases:
        if not lib.tune_checked(v):
            continue
        flags.zero_(); nxt.zero_()
        out = torch.zeros(L.n, device=dev)
        assert run(v, K, xs[0], out) == 0, name
        torch.cuda.synchronize()
        ok = (torch.equal(flags, ref_flags) and torch.equal(nxt, ref_next)
              and torch.equal(out.view(torch.int32), ref_out.view(torch.int32)))
        print(f"check {name:34s} {'ok' if ok else 'MISMATCH'}", flush=True)
        assert ok, name
    del ref_out
    scratch = torch.zeros(L.n, device=dev)  # destination of the probe that writes away from the blocks' positions
    times = {c[0]: [] for c in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 0
    for r in range(a.rounds):
        for name, v, K in cases:
            e0.record()
            for _ in range(a.reps):
                run(v, K, xs[k % 4], scratch if "contiguous" in name else xs[k % 4])
                k += 1
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) / a.reps)
    print(f"# {a.size_mib} MiB B={a.block_size} -r {a.density}: algorithmic bytes per launch {kbytes}")
    for name, _, _ in sorted(cases, key=lambda c: np.median(times[c[0]])):
        t = np.array(times[name]) * 1e-3
        print(f"{name:34s} median {np.median(t)*1e6:8.2f} us  min {t.min()*1e6:8.2f} us  "
              f"{kbytes/np.median(t)/1e9:8.1f} GB/s  frac {kbytes/np.median(t)/8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()
