#!/usr/bin/env python3
"""Round 5: per-phase timeline of the single-workgroup plan (tools/tune/plan_probe_r05.hip, generated from the product
by tools/make_plan_probe_r05.py) at config 4's mask shapes (8 workers x 4096 rows, 10 % density, 9 shard bounds).
usage: python tools/tune_plan_probe_r05.py"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "tune", "plan_probe_r05.hip")
LIB = os.path.join(ROOT, "gpurun_out", "tune", "libplan_probe_r05.so")


def main():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    t = ctypes.CDLL(LIB)
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    t.tune_plan_probe.argtypes = [vp, u32, u64, u64, u32, u32, vp, u32, vp, vp, vp, vp, ctypes.c_int, vp]
    dev = torch.device("cuda:0")
    m, rows, rpp, lanes = 8, 4096, 512, 64
    rng = np.random.default_rng(1)
    bits = rng.random((m, rows, lanes)) < 0.1
    masks = (bits.astype(np.uint64) << np.arange(lanes, dtype=np.uint64)).sum(axis=2).astype(np.uint64)
    md = torch.from_numpy(masks.view(np.int64).reshape(-1)).to(dev)
    bounds = np.array([s * rows // 8 for s in range(9)], dtype=np.int64)
    bd = torch.from_numpy(bounds).to(dev)
    wset = torch.empty(rows, dtype=torch.int64, device=dev)
    prefix = torch.empty((m + 1) * (rows + 1), dtype=torch.int32, device=dev)
    counts = torch.empty((m + 1) * 9, dtype=torch.int32, device=dev)
    tl = torch.zeros(32, dtype=torch.int64, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    names = ["masks back", "wave scans", "block scan", "stores issued"]
    for rep in range(10):
      for var in range(5):
        assert t.tune_plan_probe(md.data_ptr(), m, rows, rows, rpp, lanes, bd.data_ptr(), 9, wset.data_ptr(),
                                 prefix.data_ptr(), counts.data_ptr(), tl.data_ptr(), var, st) == 0
        torch.cuda.synchronize()
        v = tl.cpu().numpy()
        if rep < 4:
            continue
        for w, base in ((0, 0),):
            s = v[base:base + 16]
            s = s[s != 0]
            rel = [(x - s[0]) / 100.0 for x in s]  # 100 MHz -> us
            print(f"rep {rep} variant {var} wave {w:2d}: " + " ".join(f"{x:6.2f}" for x in rel), flush=True)
    print("# phases per tile:", ", ".join(names), "; last = end.  variants: 0 product, 1 no bound search, 2 no prefix "
          "stores, 3 no row stores, 4 none", flush=True)


if __name__ == "__main__":
    main()
