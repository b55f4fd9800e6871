"""How much of bench.py's timed region at --steps 20 is the host's wait for the GPU, and does a spinning wait shorten it?

The headline's timed region is K back-to-back launches of the fused scan between two torch.cuda.synchronize() calls.
Per call: (A) launches then torch.cuda.synchronize(); (B) launches, a fence-free event, a host spin on hipEventQuery
until it has completed, then torch.cuda.synchronize(); (C) as A, after hipSetDeviceFlags(hipDeviceScheduleSpin) (set
last: it changes every later wait of the process).  Each line: median and min of the host time per call and of the
host time minus the GPU span (first launch start to last end, events), 40 alternations."""
import ctypes
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

from omr import Layout, ops, timing  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
L = Layout.from_bytes(256 << 20, 256)
bm = ops.gen_bitmap(0, 0.095, L.nb)
sets = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0) for _ in range(4)]
plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
stream = torch.cuda.current_stream(dev)
launches = [plan.bind(x, x, stream) for x in sets]
hip = timing._rt()
hip.hipEventQuery.argtypes = [ctypes.c_void_p]
span = (timing.Event(), timing.Event())
tail = timing.Event()
for i in range(10):
    launches[i % 4]()
torch.cuda.synchronize()


def one(method):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    span[0].record(stream)
    for i in range(K):
        launches[i % 4]()
    span[1].record(stream)
    if method == "B":
        tail.record(stream)
        while hip.hipEventQuery(tail._e) != 0:
            pass
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e6
    g = span[0].elapsed_time(span[1]) * 1e3
    return dt, dt - g


res = {"A": [], "B": []}
for _ in range(40):
    for m in ("A", "B"):
        res[m].append(one(m))
hipDeviceScheduleSpin = 1
rc = hip.hipSetDeviceFlags(hipDeviceScheduleSpin)
res["C"] = [one("A") for _ in range(40)]
print(f"K={K} hipSetDeviceFlags(spin) rc={rc}")
for m, v in res.items():
    tot = [a for a, _ in v]
    over = [b for _, b in v]
    print(f"{m}: host us/call median {statistics.median(tot):.1f} min {min(tot):.1f} | host - gpu span median "
          f"{statistics.median(over):.1f} min {min(over):.1f} | per step {statistics.median(tot) / K:.2f}")
