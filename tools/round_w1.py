#!/usr/bin/env python3
"""The N>1 bench step's round at world 1 in a process of its own (one-rank RCCL communicator, no torch.distributed),
as bench.py's round_world1 object measures it after the headline: per-round time and the stage events.  Diagnostic
for where the N=1 anchor's time goes (e.g. run with GPU_MAX_HW_QUEUES set differently).
usage: python tools/round_w1.py [--steps 100] [--pipe defer|sync|async|thread] [--headline]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from omr import Layout, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--event-every", type=int, default=10)
    ap.add_argument("--headline", action="store_true", help="run the headline's k_scan1f launches first, as bench does")
    ap.add_argument("--pg", action="store_true",
                    help="make a one-rank torch.distributed nccl group first, as bench.py --force-dist does")
    ap.add_argument("--no-group", action="store_true",
                    help="bench.round_world1 without its own one-rank torch group (the in-process rccl1 transport)")
    # (bench.round_world1's child run reads the workload from these, as bench.py's own arguments)
    ap.add_argument("--size-mib", type=int, default=256)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29547")
        torch.cuda.set_device(0)
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    L = Layout.from_bytes(a.size_mib << 20, a.block_size)
    bm = ops.gen_bitmap(0, a.density, L.nb)
    sets = []
    for _ in range(4):
        x = ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0)
        sets.append(([x], torch.zeros(L.n, device=dev)))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    if a.headline:
        plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
        launches = [plan.bind(xs[0], xs[0], stream) for xs, _ in sets]
        for i in range(110):
            launches[i % 4]()
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = bench.round_world1(a, L, sets, dev, stream, bm, torch_group=not a.no_group)
    res["wall_s"] = round(time.perf_counter() - t0, 3)
    res["GPU_MAX_HW_QUEUES"] = os.environ.get("GPU_MAX_HW_QUEUES")
    res["headline_first"] = a.headline
    res["torch_group"] = a.pg
    res["env"] = {k: os.environ.get(k) for k in ("OMR_SIDE_QUEUES", "OMR_SIDE_PRIORITY")}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
