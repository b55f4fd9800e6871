#!/usr/bin/env python3
"""Per-workgroup timeline of one k_scan1f launch (tools/tune/fused_r02.hip "timeline" variants: the product kernel
built with ABL bit 3, which records s_memrealtime (100 MHz) at each workgroup's start, after its stream loop and
once every store it issued is acknowledged).  Prints the launch's event time next to the spread of those
timestamps, so a kernel's time above its pure read can be placed: in the streams, in the workgroups' tails, or
after the last workgroup.
usage: python tools/wg_timeline.py [--size-mib 256 --block-size 256 --density 0.095 --k 1]"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from omr import Layout, ops  # noqa: E402
from tune_r02 import load  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    torch.cuda.init()
    lib = load()
    names = {lib.tune_name(i).decode(): i for i in range(lib.tune_count())}
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.size_mib << 20, a.block_size)
    bm = ops.gen_bitmap(0, a.density, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for _ in range(4)]
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    ws = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    grid = L.num_threads * L.num_lanes * a.k
    print(f"# {a.size_mib} MiB B={a.block_size} -r {a.density} K={a.k}: {grid} workgroups", flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name in ("timeline -data-meta", "timeline -data-meta rotated", "timeline -data", "timeline product"):
        v = names[name]
        for i in range(3):  # warm-up
            lib.tune_run(v, xs[i % 4].data_ptr(), xs[i % 4].data_ptr(), flags.data_ptr(), nxt.data_ptr(),
                         ws.data_ptr(), L.n, L.block_size, a.k, 0, st)
        for r in range(a.reps):
            x = xs[(r + 3) % 4]
            ws[512 << 10:].zero_()
            torch.cuda.synchronize()
            e0.record()
            assert lib.tune_run(v, x.data_ptr(), x.data_ptr(), flags.data_ptr(), nxt.data_ptr(), ws.data_ptr(), L.n,
                                L.block_size, a.k, 0, st) == 0
            e1.record()
            torch.cuda.synchronize()
            ev_us = e0.elapsed_time(e1) * 1e3
            t = ws[512 << 10:].view(torch.int64)[:grid * 4].view(grid, 4).cpu().numpy()
            t0 = t[:, 0].min()
            start, loop, end = (t[:, 0] - t0) * TICK_US, (t[:, 1] - t0) * TICK_US, (t[:, 2] - t0) * TICK_US
            tail = end - loop
            q = lambda z: " ".join(f"{np.percentile(z, p):6.1f}" for p in (0, 10, 50, 90, 100))  # noqa: E731
            print(f"{name:22s} event {ev_us:6.1f} us | start {q(start)} | loop end {q(loop)} | acked end {q(end)} "
                  f"| tail {q(tail)}  (percentiles 0/10/50/90/100, us from the first start)", flush=True)
            if r == a.reps - 1:
                xcc = t[:, 3] & 0xF
                per = [float(end[xcc == c].max()) for c in range(8) if np.any(xcc == c)]
                print(f"{'':22s} last acked end per XCC: " + " ".join(f"{z:6.1f}" for z in per), flush=True)
                # which partition each XCC streamed (the workgroup -> column map decides it)
                cols = L.num_threads * L.num_lanes
                lin = (np.arange(grid) % 8) * (grid // 8) + np.arange(grid) // 8
                if "rotated" in name:
                    lin = (lin + grid // 8) % grid
                part = (lin // a.k) // L.num_lanes
                pp = [sorted(set(part[xcc == c].tolist())) for c in range(8)]
                print(f"{'':22s} partitions per XCC: {pp}", flush=True)


if __name__ == "__main__":
    main()
