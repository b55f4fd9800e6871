#!/usr/bin/env python3
"""Round 4: first-load latency at kernel start with 1024 waves (tools/tune/lat_r04.hip): entry-to-data time per wave
for 0 / 1 / 8 loads per lane, shared rows (as the shard sum's mask rows) or distinct rows, from a buffer that was
just written by another kernel (as the all-gathered masks are) or one read before (warm L2 / MALL).
usage: python tools/tune_lat_r04.py"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402
import torch  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "lat_r04.hip")
LIB = os.path.join(ROOT, "build", "libtune_lat_r04.so")


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp = ctypes.c_void_p
    lib.tune_lat.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint, vp, vp, vp]
    return lib


def main():
    torch.cuda.init()
    lib = load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    grid = 256  # x 4 waves = 1024 waves, one per SIMD
    stride = 1 << 20  # uint64 words between arrays (8 MiB)
    src = torch.ones(16 * stride, dtype=torch.int64, device=dev)
    tl = torch.zeros(grid * 4 * 4, dtype=torch.int64, device=dev)
    sink = torch.zeros(1, dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    print("## 1024 waves; us from the first wave's entry (p10 / p50 / p90 / max of each wave's data-back time), "
          "kernel duration by events", flush=True)
    for mode, arrays, name in ((2, 0, "no load"), (0, 1, "1 load, shared rows"), (0, 8, "8 loads, shared rows"),
                               (1, 1, "1 load, distinct rows"), (1, 8, "8 loads, distinct rows")):
        for warm in ("written just before", "read just before"):
            res, durs = [], []
            for _ in range(20):
                if warm == "written just before":
                    src.fill_(1)
                else:
                    lib.tune_lat(src.data_ptr(), stride, arrays, mode, grid, tl.data_ptr(), sink.data_ptr(), st)
                e0.record()
                assert lib.tune_lat(src.data_ptr(), stride, arrays, mode, grid, tl.data_ptr(), sink.data_ptr(), st) == 0
                e1.record()
                torch.cuda.synchronize()
                durs.append(e0.elapsed_time(e1) * 1e3)
                t = tl.view(-1, 4).cpu().numpy().astype(np.int64)
                base = t[:, 0].min()
                res.append((t[:, 1] - base) / 100.0)
            d = np.concatenate(res[2:])
            print(f"{name:24s} {warm:20s} data back p10 {np.percentile(d, 10):6.2f} p50 {np.percentile(d, 50):6.2f} "
                  f"p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f} us   kernel {np.median(durs[2:]):6.2f} us",
                  flush=True)


if __name__ == "__main__":
    main()
