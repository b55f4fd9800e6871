#!/usr/bin/env python3
"""Round 5: is the world-1 round immune to stream order now?  One process, one one-rank RCCL
communicator (optionally after a one-rank torch nccl group, as bench.py's N>1 path makes), and the round timed
(deferred reduce-scatter, out of place, 4 rotating input sets, as bench.round_world1) in four layouts, interleaved
twice:
  solo / null      the one-launch world-1 round (omr_worker_scan_tally_f32) on the caller's null stream
  solo / created   the same on a stream created after the plan
  general / null   the multi-rank round's path at world 1 (omr_dist_test_world1_round: all-gather and plan on the plan
                   stream, exchange on the exchange stream, RCCL calls): the N > 1 layout
  general / created
  general1 / ...   the same on ONE side stream (omr_ar_plan_set_side_streams(1))
Prints microseconds per round and the headline kernel's step for reference.
Round 6: the side streams are checked against the caller's stream's hardware queue before its first asynchronous round
(omr_ar_plan_queue_report is printed per cell); --no-queue-check turns the check off (round 5's behaviour).
usage: python tools/round_inproc_r05.py [--steps 200] [--reps 2] [--pipe defer|thread] [--torch-group] [--no-queue-check]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402

from omr import Layout, cdist, ops  # noqa: E402


def round_loop(eng, sets, stream, steps, thread=False):
    outs = [out for _, out in sets]
    for i in range(20):
        eng.run(sets[i % len(sets)][0][0], out=outs[i % len(sets)], mode=1, async_=True, defer=True, thread=thread)
    eng.join(stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        eng.run(sets[i % len(sets)][0][0], out=outs[i % len(sets)], mode=1, async_=True, defer=True, thread=thread)
    eng.join(stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--torch-group", action="store_true")
    ap.add_argument("--reps", type=int, default=2, help="interleaved repetitions of the four layouts")
    ap.add_argument("--pipe", choices=("defer", "thread"), default="defer",
                    help="thread: the progress thread issues the steps after the scan (host-ordered side streams)")
    ap.add_argument("--no-queue-check", action="store_true", help="side streams as made (round 5)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    if a.torch_group:
        torch.distributed.init_process_group("nccl", device_id=dev)
    L = Layout.from_bytes(256 << 20, 256)
    eng = cdist.CppSparseAllreduce(L, dev, transport="rccl1")  # (the plan and its side stream first)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    sets = []
    for _ in range(4):
        x = ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0)
        sets.append(([x], x.clone()))
    null = torch.cuda.current_stream(dev)
    created = torch.cuda.Stream(dev)
    plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
    launches = [plan.bind(xs[0], out, null) for xs, out in sets]
    res = {}
    for rep in range(a.reps):
        for layout in ("solo", "general", "general1"):
            eng.test_world1_round(layout != "solo")
            eng.replan()  # (the hook takes effect on plans made after it: general = the N>1 stream layout)
            if layout == "general1":
                eng.set_side_streams(1)  # the N>1 round's path on one side stream
            if a.no_queue_check:
                eng.set_queue_check(False)
            created = torch.cuda.Stream(dev)  # a stream created after the plan
            for sname, st in (("null", null), ("created", created)):
                with torch.cuda.stream(st):
                    us = round_loop(eng, sets, st, a.steps, thread=a.pipe == "thread")
                res.setdefault(f"{layout} / {sname}", []).append(round(us, 2))
                print(f"rep {rep} {layout:8s} {sname:8s} {us:7.2f} us per round  queues {eng.queue_report()}",
                      flush=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            launches[i % 4]()
        torch.cuda.synchronize()
        h = (time.perf_counter() - t0) / a.steps * 1e6
        res.setdefault("headline kernel (out of place)", []).append(round(h, 2))
        print(f"rep {rep} headline out of place {h:.2f} us per step", flush=True)
    eng.close()
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"torch_group": a.torch_group, "pipe": a.pipe, "queue_check": not a.no_queue_check, "steps": a.steps, "us_per_round": res}, f, indent=1)


if __name__ == "__main__":
    main()
