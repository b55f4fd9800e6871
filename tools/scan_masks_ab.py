#!/usr/bin/env python3
"""Why the world-1 round's worker scan (omr_worker_scan_f32 with `out`: flags, next, the shard sums AND the row masks,
one relaxed device atomic OR per non-zero block) takes 55 us inside the round against 47.5 us for the headline
k_scan1f (no masks): the two launches timed standalone, interleaved, on config 2's tensor (4 rotating input sets), so
the masks' atomics are separated from the round's concurrency.  Also the scan without `out` (the N>1 form).
usage: python tools/scan_masks_ab.py [--rounds 10] [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    L = Layout.from_bytes(256 << 20, 256)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0) for _ in range(4)]
    flags = torch.empty(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.empty(L.nb, dtype=torch.int32, device=dev)
    masks = torch.zeros(L.rows, dtype=torch.int64, device=dev)
    wsb = lib.omr_scan_workspace_bytes(L.n, 256, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def headline(i):  # bench's step: in place, no masks
        x = xs[i % 4]
        return lib.omr_scan_sum_fused_f32(x.data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                          nxt.data_ptr(), x.data_ptr(), ws.data_ptr(), wsb, st)

    def round_scan(i):  # the world-1 round's scan: the same + row masks (device atomics)
        x = xs[i % 4]
        return lib.omr_worker_scan_f32(x.data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                       nxt.data_ptr(), masks.data_ptr(), x.data_ptr(), ws.data_ptr(), wsb, st)

    def scan_only(i):  # the N>1 scan without the pack: masks, no sums
        x = xs[i % 4]
        return lib.omr_worker_scan_f32(x.data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                       nxt.data_ptr(), masks.data_ptr(), None, ws.data_ptr(), wsb, st)

    cases = {"headline k_scan1f (sums, no masks)": headline, "round scan (sums + masks)": round_scan,
             "scan + masks, no sums": scan_only}
    for fn in cases.values():
        assert fn(0) == 0, lib.omr_last_error().decode()
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for name, fn in cases.items():
            e0.record()
            for i in range(a.reps):
                fn(i)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times[name].append(e0.elapsed_time(e1) / a.reps * 1e3)
    for name in cases:
        print(f"{name:40s} median {np.median(times[name]):7.2f} us  (min {min(times[name]):.2f}, max {max(times[name]):.2f})",
              flush=True)


if __name__ == "__main__":
    main()
