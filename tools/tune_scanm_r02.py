#!/usr/bin/env python3
"""Round-2 study of the m-worker one-device sum (tools/tune/scanm_r02.hip): finer work units, XCD-contiguous unit
order, worker-pipelined loads, and the channel-contention test (the m worker buffers placed inside one allocation
at offsets staggered by --stagger-kib, against separate allocations).  Every variant is first checked against the
product k_scanm bit for bit (sums, flags, row masks).  Each launch is timed alone (one event pair per launch,
variants interleaved), so the spread over launches and buffer sets is visible, as in a rocprofv3 kernel trace.
Each input set has its own output tensor, as in bench.py: one output reused by every launch lets the memory-side
Infinity Cache absorb part of the 150 MB of sums written per launch, which bench.py does not get.
usage: python tools/tune_scanm_r02.py [--workers 8] [--stagger-kib sep,0,4,68] [--variants 0,2]"""
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

SRC = os.path.join(ROOT, "tools", "tune", "scanm_r02.hip")
LIB = os.path.join(ROOT, "build", "libtune_scanm_r02.so")


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_scanm.argtypes = [i, vp, u32, vp, vp, vp, u64, u32, u32, u32, vp]
    lib.tune_scanm_name.restype = ctypes.c_char_p
    return lib


def make_set(bms, L, dev, stagger):
    """The m workers' tensors: separate allocations ('sep'), or views into one allocation with worker w at
    w * (S + stagger KiB)."""
    if stagger == "sep":
        return [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for bm in bms], None
    step = L.n + int(stagger) * 256  # floats
    big = torch.empty(step * len(bms), dtype=torch.float32, device=dev)
    xs = []
    for w, bm in enumerate(bms):
        v = big[w * step:w * step + L.n]
        v.copy_(ops.fill_blocks(torch.from_numpy(bm).to(dev), L))
        xs.append(v)
    return xs, big


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=25)
    ap.add_argument("--sets", type=int, default=2, help="input sets per placement, alternated launch by launch")
    ap.add_argument("--reps", type=int, default=8, help="back-to-back launches per batch")
    ap.add_argument("--stagger-kib", default="sep")
    ap.add_argument("--variants", default="")
    ap.add_argument("--caps", default="0", help="grid caps (workgroups) for the unit kernels; 0 = a unit per wave")
    ap.add_argument("--occs", default="0", help="workgroups per CU forced with dynamic LDS (0 = registers decide)")
    a = ap.parse_args()
    torch.cuda.init()
    lib = load()
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(a.size_mib << 20, 256)
    m = a.workers
    bms = [ops.gen_bitmap(w, a.density, L.nb) for w in range(m)]
    outs = [torch.zeros(L.n, dtype=torch.float32, device=dev) for _ in range(a.sets)]  # one per set, as bench.py
    out = outs[0]
    flags = torch.zeros((m, L.nb), dtype=torch.int32, device=dev)
    masks = torch.zeros((m + 1, L.rows), dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    vids = [int(x) for x in a.variants.split(",")] if a.variants else list(range(lib.tune_scanm_count()))
    caps = [(int(c), int(o)) for c in a.caps.split(",") for o in a.occs.split(",")]
    union = np.zeros(L.nb, dtype=bool)
    for bm in bms:
        union |= bm.astype(bool)
    heads = ((np.arange(L.nb) // L.num_lanes) % L.rows_per_part) == 0
    kbytes = m * L.nbytes + int(np.count_nonzero(union | heads)) * 1024 + m * L.nb * 4 + (m + 1) * L.rows * 8
    print(f"# m={m}, {a.size_mib} MiB per worker, B=256, -r {a.density}; algorithmic bytes {kbytes}", flush=True)
    for stg in a.stagger_kib.split(","):
        sets = [make_set(bms, L, dev, stg) for _ in range(a.sets)]
        ptrs = [(ctypes.c_void_p * m)(*[x.data_ptr() for x in xs]) for xs, _ in sets]
        cases = [(v, c) for v in vids for c in (caps if v else [(0, 0)])]

        def run(v, c, k):
            return lib.tune_scanm(v, ptrs[k], m, outs[k].data_ptr(), flags.data_ptr(), masks.data_ptr(), L.n, 256,
                                  c[0], c[1], st)

        ref = None
        for v, c in cases:
            out.zero_(); flags.zero_(); masks.fill_(-1)
            assert run(v, c, 0) == 0, lib.tune_scanm_name(v)
            torch.cuda.synchronize()
            got = (out.clone(), flags.clone(), masks.clone())
            if b"ablation" in lib.tune_scanm_name(v):  # timing-only variants write a subset of the outputs
                continue
            if ref is None:
                ref = got
            else:
                ok = all(torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x, y.view(torch.int32)
                                     if y.dtype == torch.float32 else y) for x, y in zip(ref, got))
                assert ok, f"{lib.tune_scanm_name(v).decode()} cap {c}: mismatch vs the product"
        del ref, got
        times = {vc: [[] for _ in range(a.sets)] for vc in cases}
        # per round and case: --reps launches back to back (sets alternating, as bench rotates them), every launch
        # between its own pair of events, one synchronisation at the end of the batch
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
        for r in range(a.rounds):
            for vc in cases:
                for j in range(a.reps):
                    evs[j][0].record()
                    run(vc[0], vc[1], j % a.sets)
                    evs[j][1].record()
                torch.cuda.synchronize()
                if r:
                    for j in range(a.reps):
                        times[vc][j % a.sets].append(evs[j][0].elapsed_time(evs[j][1]))
        print(f"## placement {stg}{'' if stg == 'sep' else ' KiB stagger in one allocation'}", flush=True)
        for vc in sorted(cases, key=lambda vc: np.median(np.concatenate(times[vc]))):
            t = np.concatenate(times[vc]) * 1e-3
            per = " ".join(f"{np.median(x) * 1e3:7.2f}" for x in times[vc])
            nm = (lib.tune_scanm_name(vc[0]).decode() + (f" cap{vc[1][0]}" if vc[1][0] else "") +
                  (f" occ{vc[1][1]}" if vc[1][1] else ""))
            print(f"{nm:32s} median {np.median(t)*1e6:8.2f} us  min {t.min()*1e6:8.2f}  max {t.max()*1e6:8.2f}  "
                  f"spread {t.max()/t.min()-1:6.1%}  frac {kbytes/np.median(t)/8e12:.4f}  per set {per}", flush=True)
        del sets, ptrs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
