#!/usr/bin/env python3
"""Round 4: does the world-1 round still run 2.3x slower when its one-rank RCCL communicator is made inside a process
that has already run the headline (bench.py's round_world1 with torch_group=False)?  Round 3 measured
118-154 us per round that way against 59 us under torch.distributed.run, with RCCL's own streams issuing fill and
copy kernels every round.  Since round 4 a one-rank group's collectives are plain copies (no RCCL call per round).
This runs the headline loop for a while (as bench.py does), then the in-process round, and prints both.
usage: python tools/round_inproc_r04.py [--steps 200]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from omr import Layout, ops  # noqa: E402


def round_loop(eng, sets, stream, steps):
    """bench.round_world1's loop on a given engine: reduce-scatter, deferred, out of place; us per round."""
    outs = []
    for xs, out in sets:
        out.copy_(xs[0])
        outs.append(out)
    for i in range(20):
        eng.run(sets[i % len(sets)][0][0], out=outs[i % len(sets)], mode=1, async_=True, defer=True)
    eng.join(stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.run(sets[i % len(sets)][0][0], out=outs[i % len(sets)], mode=1, async_=True, defer=True)
    eng.join(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--comm-first", action="store_true",
                    help="make the one-rank communicator and plan before any kernel runs, then the headline, then the "
                         "round on that plan")
    ap.add_argument("--torch-group", action="store_true", help="--comm-first after a one-rank torch nccl group")
    a = ap.parse_args()
    if a.comm_first:
        from omr import cdist
        args = bench.parse(["--no-cpu"])
        dev = torch.device("cuda:0")
        if a.torch_group:  # a one-rank torch nccl group first, as bench.py's N>1 path makes (env: MASTER_*, RANK, ...)
            before = dict(os.environ)
            torch.cuda.set_device(0)
            torch.distributed.init_process_group("nccl", device_id=dev)
            changed = {k: v for k, v in os.environ.items() if before.get(k) != v}
            print(f"torch group made; environment it changed: {changed}", flush=True)
        L = Layout.from_bytes(args.size_mib << 20, args.block_size)
        eng = cdist.CppSparseAllreduce(L, dev, transport="rccl1")  # (first GPU work of the process)
        bm = ops.gen_bitmap(0, args.density, L.nb)
        sets = [([ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0)], torch.zeros(L.n, device=dev))
                for _ in range(4)]
        stream = torch.cuda.current_stream(dev)
        print(f"comm first, round before the headline: {round_loop(eng, sets, stream, a.steps):.1f} us", flush=True)
        side = torch.cuda.Stream(dev)  # the same rounds issued on a created (non-null) stream
        with torch.cuda.stream(side):
            print(f"comm first, round on a created stream: {round_loop(eng, sets, side, a.steps):.1f} us "
                  f"(stream {side.cuda_stream:#x}; null stream {stream.cuda_stream:#x})", flush=True)
        plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
        launches = [plan.bind(xs[0], xs[0], stream) for xs, _ in sets]
        for i in range(a.steps):
            launches[i % 4]()
        torch.cuda.synchronize()
        print(f"comm first, round after the headline: {round_loop(eng, sets, stream, a.steps):.1f} us", flush=True)
        eng.close()
        return
    args = bench.parse(["--no-cpu", "--steps", str(a.steps), "--warmup", "20"])
    dev = torch.device("cuda:0")
    L = Layout.from_bytes(args.size_mib << 20, args.block_size)
    bm = ops.gen_bitmap(0, args.density, L.nb)
    sets = [([ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0)], torch.zeros(L.n, device=dev))
            for _ in range(4)]
    stream = torch.cuda.current_stream(dev)
    plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
    launches = [plan.bind(xs[0], xs[0], stream) for xs, _ in sets]
    for i in range(50):
        launches[i % 4]()
    torch.cuda.synchronize()
    def headline(what):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            launches[i % 4]()
        torch.cuda.synchronize()
        print(f"headline {what}: {(time.perf_counter() - t0) / a.steps * 1e6:.2f} us per step", flush=True)

    headline("before any communicator")
    # a one-rank communicator made here, then the headline again: does making it slow down every kernel?
    from omr import cdist
    eng = cdist.CppSparseAllreduce(L, dev, transport="rccl1")
    headline("after a one-rank RCCL communicator was made")
    eng.close()
    headline("after it was destroyed")
    for k in range(2):
        r = bench.round_world1(args, L, sets, dev, stream, bm, torch_group=False)
        print(f"in-process round {k}: {r['ms_per_round'] * 1e3:.1f} us per round, scan {r['scan_in_round']}", flush=True)
        headline(f"after in-process round {k}")


if __name__ == "__main__":
    main()
