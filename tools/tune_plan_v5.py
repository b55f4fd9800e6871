#!/usr/bin/env python3
"""Round 5: where the row-chunk plan's 6-8 us at config 4's shapes go (<= 6 us).  The round's own
call (no union stored, no chain, own masks and pack counters cleared, shard 0's pair list, counts tagged) in the study
variants of tools/tune/plan_v5_study.hip, with the counts in pinned host memory (as the round) and in device memory,
and without the pair list.  Outputs of every exact variant checked against the product's.  Run under rocprofv3
--kernel-trace: the kernel names carry the variant (k_round_plan_study<W, V>); the log gives the order of the cases.
usage: python tools/tune_plan_v5.py [--reps 50] [--rounds 3]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import _lib  # noqa: E402
import tune_round_r03 as r03  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "plan_v5_study.hip")
LIB = os.path.join(ROOT, "tools", "tune", "libplan_v5.so")  # built here before the GPU call (git-ignored)
VARIANTS = {0: "product form", 1: "speculative loads", 2: "no ticket", 3: "no wait (timing only)",
            4: "speculative loads, polls without sleep"}


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    t = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    t.tune_plan_v5.argtypes = [i, vp, u32, u64, u64, u32, u32, vp, u32, vp, vp, vp, vp, vp, vp, u32, vp, u32, u32, vp,
                               vp]
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--workers", type=int, default=8)
    a = ap.parse_args()
    a.only = ""
    torch.cuda.init()
    t = load()
    lib = _lib.load()
    D = r03.setup(a)
    L, m, naggs, rows, B, NB, mstride = (D[k] for k in ("L", "m", "naggs", "rows", "B", "NB", "mstride"))
    masks_all, bdev, roff, st, dev = D["masks_all"], D["bdev"], D["roff"], D["st"], D["dev"]
    r0, r1 = D["r0"], D["r1"]
    units, cap = ctypes.c_uint64(), ctypes.c_uint32()
    _lib.check(lib.omr_sum_list_geometry(L.n, B, NB, L.num_threads, r0, r1, m, ctypes.byref(units), ctypes.byref(cap)),
               "geometry")
    lrec = torch.empty(units.value * cap.value, dtype=torch.int64, device=dev)
    lcnt = torch.empty(units.value, dtype=torch.int32, device=dev)
    sl = _lib.SumList(lrec.data_ptr(), lcnt.data_ptr(), r0, r1, 2 * rows, 0)
    for w in range(m):
        sl.recv_offsets[w] = int(roff[w])
    pin = torch.zeros(4096, dtype=torch.int64).pin_memory()
    pin_d = ctypes.c_void_p()
    assert ctypes.CDLL("libamdhip64.so").hipHostGetDevicePointer(ctypes.byref(pin_d), ctypes.c_void_p(pin.data_ptr()),
                                                                 0) == 0
    dcnt = torch.zeros(4096, dtype=torch.int64, device=dev)
    zmask = torch.empty(rows, dtype=torch.int64, device=dev)
    zcnt = torch.empty(naggs, dtype=torch.int32, device=dev)
    wset = torch.empty(rows, dtype=torch.int64, device=dev)
    prefix = torch.empty((m + 1) * (rows + 1), dtype=torch.int32, device=dev)
    ws = torch.zeros(int(lib.omr_round_plan_workspace_words()), dtype=torch.int64, device=dev)
    seq = [0]
    ncnt = (m + 1) * (naggs + 1)

    def call(v, counts_ptr, with_list):
        seq[0] += 1
        if v is None:  # the product
            return lib.omr_round_plan_list(masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB,
                                           bdev.data_ptr(), naggs + 1, wset.data_ptr(), None, prefix.data_ptr(),
                                           counts_ptr, zmask.data_ptr(), zcnt.data_ptr(), naggs, ws.data_ptr(),
                                           seq[0], None, B, ctypes.byref(sl) if with_list else None, st)
        return t.tune_plan_v5(v, masks_all.data_ptr(), m, mstride, rows, L.rows_per_part, NB, bdev.data_ptr(),
                              naggs + 1, wset.data_ptr(), None, prefix.data_ptr(), counts_ptr, zmask.data_ptr(),
                              zcnt.data_ptr(), naggs, ws.data_ptr(), seq[0], B, ctypes.byref(sl) if with_list else None,
                              st)

    # reference outputs from the product
    assert call(None, dcnt.data_ptr(), True) == 0, lib.omr_last_error()
    torch.cuda.synchronize()
    ref = (wset.clone(), prefix.clone(), dcnt[:ncnt].clone() & 0xFFFFFFFF, lrec.clone(), lcnt.clone())
    for v in VARIANTS:
        if v == 3:
            continue
        for c in (pin_d.value, dcnt.data_ptr()):
            wset.zero_(), prefix.zero_(), lrec.zero_(), lcnt.zero_()
            assert call(v, c, True) == 0
            torch.cuda.synchronize()
            got_c = (torch.from_numpy(pin.numpy()[:ncnt].copy()).to(dev) if c == pin_d.value else dcnt[:ncnt])
            assert int((got_c >> 32)[0].item()) == seq[0], f"variant {v}: counts not tagged"
            got = (wset, prefix, got_c & 0xFFFFFFFF, lrec, lcnt)
            for x, y, n in zip(got, ref, ("write set", "prefix", "counts", "records", "record counts")):
                assert torch.equal(x, y), f"variant {v}: {n} differs"
    print("# every exact variant == the product", flush=True)
    cases = []
    for with_list in (True, False):
        for where, c in (("pinned", pin_d.value), ("device", dcnt.data_ptr())):
            cases.append((f"product, {'list' if with_list else 'no list'}, counts {where}", None, c, with_list))
            for v, name in VARIANTS.items():
                cases.append((f"V{v} {name}, {'list' if with_list else 'no list'}, counts {where}", v, c, with_list))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {n: [] for n, *_ in cases}
    for r in range(a.rounds):
        for name, v, c, wl in cases:
            print(f"# case {name}", flush=True)
            e0.record()
            for _ in range(a.reps):
                call(v, c, wl)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) * 1e3 / a.reps)
    for name, *_ in cases:
        print(f"{name:64s} {np.median(res[name]):7.2f} us per launch by events (host-bound below ~10 us)")


if __name__ == "__main__":
    main()
