#!/usr/bin/env python3
"""PCIe probe for the host-resident path: one pinned-host <-> HBM link, H2D alone, D2H alone, and both directions at
once on two streams (what the staged bucket pipeline of omr_sparse_buckets_f32 needs: bucket k+1 in while bucket k-2
goes out).  usage: python tools/pcie_duplex.py [--mib 256]"""
import argparse
import json

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = (a.mib << 20) // 4
    h_in = torch.ones(n).pin_memory()
    h_out = torch.zeros(n).pin_memory()
    d_in = torch.empty(n, device="cuda")
    d_out = torch.ones(n, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}

    def timed(fn):
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            torch.cuda.current_stream().wait_stream(s1)
            torch.cuda.current_stream().wait_stream(s2)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e-3)
        return best

    def h2d():
        s1.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            d_in.copy_(h_in, non_blocking=True)

    def d2h():
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            h_out.copy_(d_out, non_blocking=True)

    nbytes = n * 4
    t = timed(h2d)
    res["h2d_GBps"] = round(nbytes / t / 1e9, 2)
    t = timed(d2h)
    res["d2h_GBps"] = round(nbytes / t / 1e9, 2)
    t = timed(lambda: (h2d(), d2h()))
    res["both_directions_GBps_each"] = round(nbytes / t / 1e9, 2)
    res["both_directions_GBps_total"] = round(2 * nbytes / t / 1e9, 2)
    res["mib"] = a.mib
    print(json.dumps(res))


if __name__ == "__main__":
    main()
