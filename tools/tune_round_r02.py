#!/usr/bin/env python3
"""The multi-rank round's aggregator-side kernels at config-4 shapes on one MI355X (tools/tune/round_r02.hip): the
shard sum of shard 0 of 8 with 8 workers' contributions (8 x 256 MiB, -r 0.095, worker 0 aggregating, its own
blocks read in place), and the world-1 shard sum (the whole tensor, one worker); the product's k_shard_sum against
variants that issue every contributor's loads at once; plus the product's pack (k_move) of worker 0's blocks of
the other shards.  Variants are checked against the product bit for bit.  Batch-timed, interleaved.
usage: python tools/tune_round_r02.py [--workers 8] [--rounds 10]"""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, _lib, ops  # noqa: E402

SRC = os.path.join(ROOT, "tools", "tune", "round_r02.hip")
LIB = os.path.join(ROOT, "build", "libtune_round_r02.so")


def load():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-I" + os.path.join(ROOT, "include"), "-o", LIB, SRC], check=True)
    lib = ctypes.CDLL(LIB)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.tune_shard_sum.argtypes = [i, vp, u32, vp, vp, vp, u32, vp, vp, u64, u64, u64, u32, i, vp, u32, vp]
    lib.tune_name.restype = ctypes.c_char_p
    lib.tune_max_count.restype = u32
    lib.tune_move.argtypes = [i, vp, vp, vp, vp, u64, u32, u64, u64, u32, u32, vp]
    lib.tune_move_name.restype = ctypes.c_char_p
    return lib


def setup(L, m, naggs, dev, stream):
    """m workers' tensors, their masks (omr_scan_f32), the round plan over them, and shard 0's received streams
    (workers 1.. packed over shard 0's rows, as the exchange would deliver them)."""
    lib = _lib.load()
    xs = [ops.fill_blocks(torch.from_numpy(ops.gen_bitmap(w, 0.095, L.nb)).to(dev), L) for w in range(m)]
    masks = torch.zeros((m, L.rows), dtype=torch.int64, device=dev)
    flags = torch.empty(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.empty(L.nb, dtype=torch.int32, device=dev)
    for w in range(m):
        _lib.check(lib.omr_scan_f32(xs[w].data_ptr(), L.n, 256, L.num_lanes, L.num_threads, flags.data_ptr(),
                                    masks[w].data_ptr(), nxt.data_ptr(), stream), "omr_scan_f32")
    bounds = [s * L.rows // naggs for s in range(naggs + 1)]
    bdev = torch.tensor(bounds, dtype=torch.int64, device=dev)
    wset = torch.empty(L.rows, dtype=torch.int64, device=dev)
    umask = torch.empty(L.rows, dtype=torch.int64, device=dev)
    prefix = torch.empty((m + 1, L.rows + 1), dtype=torch.int32, device=dev)
    counts = torch.empty((m + 1, naggs + 1), dtype=torch.int64, device=dev)
    pws = torch.zeros(int(lib.omr_round_plan_workspace_words()), dtype=torch.int64, device=dev)
    _lib.check(lib.omr_round_plan(masks.data_ptr(), m, L.rows, L.rows_per_part, L.num_lanes, bdev.data_ptr(),
                                  naggs + 1, wset.data_ptr(), umask.data_ptr(), prefix.data_ptr(), counts.data_ptr(),
                                  None, pws.data_ptr(), 1, stream), "omr_round_plan")
    torch.cuda.synchronize()
    cnt = counts.cpu().numpy() & 0xFFFFFFFF  # ((seq << 32) | count)
    r0, r1 = bounds[0], bounds[1]
    per = [int(cnt[c, 1] - cnt[c, 0]) for c in range(m)]
    recv_off = np.zeros(m, dtype=np.uint64)
    acc = 0
    for c in range(1, m):
        recv_off[c] = acc
        acc += per[c]
    recv = torch.empty(max(acc, 1) * 256, dtype=torch.float32, device=dev)
    for c in range(1, m):  # worker c's shard-0 stream: its blocks of rows [r0, r1), others skipped
        _lib.check(lib.omr_move_blocks_f32(xs[c].data_ptr(), recv[int(recv_off[c]) * 256:].data_ptr(), 0,
                                           masks[c].data_ptr(), prefix[c].data_ptr(), L.rows, L.num_lanes, 256, r1,
                                           L.rows, stream), "pack")
    torch.cuda.synchronize()
    return dict(xs=xs, masks=masks, prefix=prefix, wset=wset, recv=recv, recv_off=recv_off, r0=r0, r1=r1,
                bounds=bounds, union_blocks=int(cnt[m, 1] - cnt[m, 0]), contributions=sum(per))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--lgs", default="0", help="lanes per unit (0 = the product's choice)")
    a = ap.parse_args()
    torch.cuda.init()
    tl = load()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    L = Layout.from_bytes(256 << 20, 256)
    lgs = [int(x) for x in a.lgs.split(",")]
    for m, naggs, label in [(a.workers, a.workers, f"shard 0 of {a.workers}, {a.workers} workers"),
                            (1, 1, "world 1: whole tensor, one worker")]:
        S = setup(L, m, naggs, dev, st)
        r0, r1 = S["r0"], S["r1"]
        roff = (ctypes.c_uint64 * m)(*[int(v) for v in S["recv_off"]])
        out_ref = S["xs"][0].clone()
        outs = {}
        cases = [(v, lg) for v in range(tl.tune_count()) if m <= tl.tune_max_count(v) for lg in lgs]

        def run(v, lg, out):
            return tl.tune_shard_sum(v, S["xs"][0].data_ptr(), 0, S["recv"].data_ptr(), roff, S["masks"].data_ptr(),
                                     m, S["prefix"].data_ptr(), S["wset"].data_ptr(), L.rows, r0, r1, L.num_lanes, 0,
                                     out.data_ptr(), lg, st)

        for v, lg in cases:
            o = S["xs"][0].clone()
            assert run(v, lg, o) == 0, tl.tune_name(v)
            torch.cuda.synchronize()
            outs[(v, lg)] = o
        ref = outs[cases[0]]
        for k, o in outs.items():
            assert torch.equal(o.view(torch.int32), ref.view(torch.int32)), f"{tl.tune_name(k[0]).decode()} mismatch"
        del outs
        packed = torch.empty(L.n, dtype=torch.float32, device=dev)
        work = [S["xs"][0].clone() for _ in range(2)]
        times = {c: [] for c in cases}
        times["pack"] = []
        mcases = [(v, lg, g) for v in range(tl.tune_move_count()) for lg in (0, 16, 64) for g in (0, 1024, 4096)]
        for mc in mcases:
            times[mc] = []
        ref_pack = torch.zeros(L.n, dtype=torch.float32, device=dev)
        lib.omr_move_blocks_f32(S["xs"][0].data_ptr(), ref_pack.data_ptr(), 0, S["masks"][0].data_ptr(),
                                S["prefix"][0].data_ptr(), L.rows, L.num_lanes, 256, r0, r1, st)
        for v, lg, g in mcases:
            chk = torch.zeros(L.n, dtype=torch.float32, device=dev)
            assert tl.tune_move(v, S["xs"][0].data_ptr(), chk.data_ptr(), S["masks"][0].data_ptr(),
                                S["prefix"][0].data_ptr(), L.rows, L.num_lanes, r0, r1, lg, g, st) == 0
            torch.cuda.synchronize()
            assert torch.equal(chk.view(torch.int32), ref_pack.view(torch.int32)), tl.tune_move_name(v)
        del chk, ref_pack
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for r in range(a.rounds):
            for c in cases:
                e0.record()
                for i in range(a.reps):
                    run(c[0], c[1], work[i % 2])
                e1.record()
                torch.cuda.synchronize()
                if r:
                    times[c].append(e0.elapsed_time(e1) / a.reps)
            e0.record()
            for i in range(a.reps):  # worker 0's pack of the other shards (its own shard skipped)
                lib.omr_move_blocks_f32(S["xs"][0].data_ptr(), packed.data_ptr(), 0, S["masks"][0].data_ptr(),
                                        S["prefix"][0].data_ptr(), L.rows, L.num_lanes, 256, r0, r1, st)
            e1.record()
            torch.cuda.synchronize()
            if r:
                times["pack"].append(e0.elapsed_time(e1) / a.reps)
            for mc in mcases:
                e0.record()
                for i in range(a.reps):
                    tl.tune_move(mc[0], S["xs"][0].data_ptr(), packed.data_ptr(), S["masks"][0].data_ptr(),
                                 S["prefix"][0].data_ptr(), L.rows, L.num_lanes, r0, r1, mc[1], mc[2], st)
                e1.record()
                torch.cuda.synchronize()
                if r:
                    times[mc].append(e0.elapsed_time(e1) / a.reps)
        ub, nc = S["union_blocks"], S["contributions"]
        own_blocks = int(sum(bin(int(x) & 0xFFFFFFFFFFFFFFFF).count("1") for x in S["masks"][0][r0:r1].cpu().numpy()))
        sbytes = (nc + own_blocks + ub) * 1024
        print(f"## {label}: write-set blocks {ub}, received contributions {nc}, own {own_blocks}: "
              f"{sbytes} algorithmic bytes", flush=True)
        for c in sorted(cases, key=lambda c: np.median(times[c])):
            t = np.median(times[c]) * 1e-3
            print(f"{tl.tune_name(c[0]).decode():28s} lg {c[1] or 'auto':>4}  median {t * 1e6:8.2f} us  "
                  f"{sbytes / t / 1e9:7.1f} GB/s", flush=True)
        pb = S["masks"][0].cpu().numpy()
        tot = int(sum(bin(int(x) & 0xFFFFFFFFFFFFFFFF).count("1") for x in pb)) - own_blocks
        t = np.median(times["pack"]) * 1e-3
        print(f"{'product pack (k_move)':28s}           median {t * 1e6:8.2f} us  {2 * tot * 1024 / t / 1e9:7.1f} GB/s "
              f"({tot} blocks read + written)", flush=True)
        for mc in sorted(mcases, key=lambda mc: np.median(times[mc]))[:8]:
            t = np.median(times[mc]) * 1e-3
            print(f"  {tl.tune_move_name(mc[0]).decode():26s} lg {mc[1] or 'auto':>4} grid {mc[2] or 'auto':>5}  "
                  f"median {t * 1e6:8.2f} us  {2 * tot * 1024 / t / 1e9:7.1f} GB/s", flush=True)
        del S, work, packed
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
