#!/usr/bin/env python3
"""Time the m-worker one-device sum (k_scanm, the product's launch for m >= 2) against k_scanm2 shapes, side by
side in one process with bench-style batch timing (one event pair around --reps launches); every variant's sums,
flags and masks are checked bit-exactly against the product's first.
usage: python tools/tune_scanm.py [--workers 8] [--rounds 8]"""
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

SRC = os.path.join(ROOT, "omnireduce-rdma-demo_amd", "csrc", "tune", "scanm_variants.hip")
LIB = os.path.join(ROOT, "build", "libtune_scanm.so")


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_scanm.argtypes = [i, vp, u32, vp, vp, vp, u64, u32, vp]
    lib.tune_scanm_name.restype = ctypes.c_char_p
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10, help="launches between one pair of events")
    a = ap.parse_args()
    torch.cuda.init()
    lib = build()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.size_mib << 20, a.block_size)
    m = a.workers
    bms = [ops.gen_bitmap(w, a.density, L.nb) for w in range(m)]
    sets = [[ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for bm in bms] for _ in range(2)]
    ptrs = [(ctypes.c_void_p * m)(*[x.data_ptr() for x in xs]) for xs in sets]
    out = torch.zeros(L.n, dtype=torch.float32, device=dev)
    flags = torch.zeros((m, L.nb), dtype=torch.int32, device=dev)
    masks = torch.zeros((m + 1, L.rows), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def run(v, k):
        return lib.tune_scanm(v, ptrs[k], m, out.data_ptr(), flags.data_ptr(), masks.data_ptr(), L.n, L.block_size,
                              st)

    ref = None
    for v in range(lib.tune_scanm_count()):
        out.zero_()
        flags.zero_()
        masks.zero_()
        assert run(v, 0) == 0, lib.tune_scanm_name(v)
        torch.cuda.synchronize()
        got = (out.clone(), flags.clone(), masks.clone())
        if ref is None:
            ref = got
        else:
            assert all(torch.equal(x, y) for x, y in zip(ref, got)), lib.tune_scanm_name(v).decode()
    union = np.zeros(L.nb, dtype=bool)
    for bm in bms:
        union |= bm.astype(bool)
    heads = ((np.arange(L.nb) // L.num_lanes) % L.rows_per_part) == 0
    kbytes = m * L.nbytes + int(np.count_nonzero(union | heads)) * L.block_size * 4 + m * L.nb * 4 + \
        (m + 1) * L.rows * 8
    times = {v: [] for v in range(lib.tune_scanm_count())}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    k = 0
    for r in range(a.rounds):
        for v in times:
            e0.record()
            for _ in range(a.reps):
                run(v, k % 2)
                k += 1
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[v].append(e0.elapsed_time(e1) / a.reps)
    print(f"# m={m}, {a.size_mib} MiB per worker, B={a.block_size}, -r {a.density}; algorithmic bytes {kbytes}")
    for v in sorted(times, key=lambda v: np.median(times[v])):
        t = np.median(times[v]) * 1e-3
        print(f"{lib.tune_scanm_name(v).decode():22s} median {t * 1e6:8.2f} us  {kbytes / t / 1e9:8.1f} GB/s "
              f"({kbytes / t / 8e12:.3f} of 8 TB/s)")


if __name__ == "__main__":
    main()
