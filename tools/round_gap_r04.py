#!/usr/bin/env python3
"""Round 4: where the world-1 round's 4.5-11 us gap between consecutive worker scans comes from.  The kernel traces
(profiles/r04/round_w1_trace/, gpurun_out r4k) show the scans issued 35-70 us ahead of time, yet each starts 4.5-11 us
after the previous one ends, while back-to-back headline launches leave no gap.  Here the round's scan is launched
back to back on one stream, adding one ingredient of the round at a time, each case batch-timed with events
(per-launch mean; 4 rotating input sets), interleaved:
  A  headline k_scan1f, in place
  B  the round's scan (+ row masks), in place
  C  the round's scan, out of place (sums into a separate buffer, as the round writes `out`)
  D  C + an event record after every scan (the round's `scanned`: DisableTiming | DisableSystemFence)
  E  D + a side stream that waits for each record and copies 32 KiB (the world-1 all-gather)
  F  E + a device-to-host-mapped 4-byte write on the side stream (hipMemsetAsync of a pinned word: the count notice)
  G  C + a stream write of a sequence number after every scan (hipStreamWriteValue32 to signal memory), no event
  H  G + a side stream that waits for it (hipStreamWaitValue32 >=) and copies 32 KiB
usage: python tools/round_gap_r04.py [--rounds 8] [--reps 20]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, _lib, ops  # noqa: E402

EV_FLAGS = 0x2 | 0x20000000  # hipEventDisableTiming | hipEventDisableSystemFence (omr_dist.hip's round events)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    lib = _lib.load()
    hip = ctypes.CDLL("libamdhip64.so")
    vp = ctypes.c_void_p
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    hip.hipEventRecord.argtypes = [vp, vp]
    hip.hipStreamWaitEvent.argtypes = [vp, vp, ctypes.c_uint]
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    hip.hipMemsetAsync.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, vp]
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t, ctypes.c_uint]
    hip.hipStreamWriteValue32.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint]
    hip.hipStreamWaitValue32.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
    sig = vp()
    assert hip.hipExtMallocWithFlags(ctypes.byref(sig), 8, 0x2) == 0  # hipMallocSignalMemory
    seq = [0]
    evs = []
    for _ in range(3):
        e = vp()
        assert hip.hipEventCreateWithFlags(ctypes.byref(e), EV_FLAGS) == 0
        evs.append(e)
    L = Layout.from_bytes(256 << 20, 256)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0) for _ in range(4)]
    outs = [x.clone() for x in xs]
    flags = torch.empty(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.empty(L.nb, dtype=torch.int32, device=dev)
    masks = torch.zeros(L.rows, dtype=torch.int64, device=dev)
    gathered = torch.zeros(L.rows, dtype=torch.int64, device=dev)
    pinned = torch.zeros(16, dtype=torch.int32).pin_memory()
    wsb = lib.omr_scan_workspace_bytes(L.n, 256, L.num_lanes, L.num_threads)
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream(dev)
    ss = side.cuda_stream

    def scan(i, place, msk=True):
        x = xs[i % 4]
        o = x if place else outs[i % 4]
        return lib.omr_worker_scan_f32(x.data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                       nxt.data_ptr(), masks.data_ptr() if msk else None, o.data_ptr(), ws.data_ptr(),
                                       wsb, st)

    def A(i):
        x = xs[i % 4]
        return lib.omr_scan_sum_fused_f32(x.data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                          nxt.data_ptr(), x.data_ptr(), ws.data_ptr(), wsb, st)

    def B(i):
        return scan(i, True)

    def C(i):
        return scan(i, False)

    def D(i):
        rc = scan(i, False)
        return rc or hip.hipEventRecord(evs[i % 3], st)

    def E(i):
        rc = D(i)
        rc = rc or hip.hipStreamWaitEvent(ss, evs[i % 3], 0)
        return rc or hip.hipMemcpyAsync(gathered.data_ptr(), masks.data_ptr(), 32 << 10, 3, ss)

    def F(i):
        rc = E(i)
        return rc or hip.hipMemsetAsync(pinned.data_ptr(), 0, 4, ss)

    def G(i):
        rc = scan(i, False)
        seq[0] += 1
        return rc or hip.hipStreamWriteValue32(st, sig, seq[0], 0)

    def H(i):
        rc = G(i)
        rc = rc or hip.hipStreamWaitValue32(ss, sig, seq[0], 0x0, 0xFFFFFFFF)  # hipStreamWaitValueGte
        return rc or hip.hipMemcpyAsync(gathered.data_ptr(), masks.data_ptr(), 32 << 10, 3, ss)

    cases = {"A headline, in place": A, "B round scan (+ masks), in place": B, "C round scan, out of place": C,
             "D C + event record per scan": D, "E D + side stream: wait + 32 KiB copy": E,
             "F E + side-stream pinned 4-byte memset": F, "G C + stream write value per scan": G,
             "H G + side stream: wait value + 32 KiB copy": H}
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
    print(f"## config 2's tensor (256 MiB, B=256, -r 0.095), {a.reps} launches per batch, per-launch mean", flush=True)
    for name in cases:
        print(f"{name:44s} median {np.median(times[name]):7.2f} us  (min {min(times[name]):.2f}, "
              f"max {max(times[name]):.2f})", flush=True)


if __name__ == "__main__":
    main()
