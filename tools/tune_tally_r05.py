#!/usr/bin/env python3
"""Round 5: the one-launch world-1 round's scan (omr_worker_scan_tally_f32) against the headline kernel
(omr_scan_sum_fused_f32) at config 2 (256 MiB, B=256, -r 0.095), launched back to back from pre-converted ctypes
arguments (no round driver): in place and out of place, the tally alone, the tally with workgroup 0 publishing the
previous launch's counts.  Batch-timed with events over 100 launches, 4 rotating buffers, interleaved 3 times.
usage: python tools/tune_tally_r05.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, _lib, ops  # noqa: E402


def main():
    lib = _lib.load()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(256 << 20, 256)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for _ in range(4)]
    outs = [x.clone() for x in xs]
    flags = torch.empty(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.empty(L.nb, dtype=torch.int32, device=dev)
    wsb = lib.omr_scan_workspace_bytes(L.n, 256, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    slots = lib.omr_tally_slots(L.n, 256, L.num_lanes, L.num_threads)
    tally = torch.zeros(4 * slots, dtype=torch.int64, device=dev)
    pin = torch.zeros(64, dtype=torch.int32).pin_memory()
    pd = ctypes.c_void_p()
    assert ctypes.CDLL("libamdhip64.so").hipHostGetDevicePointer(ctypes.byref(pd), ctypes.c_void_p(pin.data_ptr()), 0) == 0
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    seq = [0]

    def headline(i, inplace):
        o = xs[i % 4] if inplace else outs[i % 4]
        return lib.omr_scan_sum_fused_f32(P(xs[i % 4]), L.n, 256, L.num_lanes, L.num_threads, P(flags), P(nxt), P(o),
                                          P(ws), wsb, st)

    def tally_scan(i, inplace, publish):
        o = xs[i % 4] if inplace else outs[i % 4]
        k, kp = i % 4, (i - 1) % 4
        seq[0] += 1
        return lib.omr_worker_scan_tally_f32(P(xs[i % 4]), L.n, 256, L.num_lanes, L.num_threads, P(flags), P(nxt),
                                             P(o), ctypes.c_void_p(tally.data_ptr() + 8 * slots * k),
                                             ctypes.c_void_p(tally.data_ptr() + 8 * slots * kp) if publish else None,
                                             ctypes.c_void_p(pd.value + 16 * kp) if publish else None, seq[0], P(ws),
                                             wsb, st)

    cases = {"headline in place": lambda i: headline(i, True), "headline out of place": lambda i: headline(i, False),
             "tally in place": lambda i: tally_scan(i, True, False),
             "tally out of place": lambda i: tally_scan(i, False, False),
             "tally + publish, out of place (the one-launch round)": lambda i: tally_scan(i, False, True)}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {k: [] for k in cases}
    for r in range(4):
        for name, fn in cases.items():
            for i in range(10):
                assert fn(i) == 0, lib.omr_last_error()
            e0.record()
            for i in range(100):
                fn(i)
            e1.record()
            torch.cuda.synchronize()
            if r:
                res[name].append(e0.elapsed_time(e1) / 100 * 1e3)
    for name, v in res.items():
        print(f"{name:55s} {np.median(v):7.2f} us  ({', '.join(f'{x:.2f}' for x in v)})", flush=True)


if __name__ == "__main__":
    main()
