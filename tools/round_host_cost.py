#!/usr/bin/env python3
"""Host cost of one multi-rank round call (omr_sparse_round_f32 through omr/cdist.py) at world 1 over RCCL, per
pipeline mode: wall time of each call on the host, next to the GPU period of the same loop.  The round is
host-bound when the call takes longer than the worker scan it queues.
usage: python tools/round_host_cost.py [--rounds 300] [--modes sync,async,defer]"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from omr import Layout, cdist, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--modes", default="sync,async,defer")
    ap.add_argument("--size-mib", type=int, default=256)
    a = ap.parse_args()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29517"), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    L = Layout.from_bytes(a.size_mib << 20, 256)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L) for _ in range(4)]
    outs = [x.clone() for x in xs]
    eng = cdist.CppSparseAllreduce(L, dev)
    st = torch.cuda.current_stream(dev)
    for mode in a.modes.split(","):
        kw = dict(mode=1, async_=mode != "sync", defer=mode == "defer")
        for i in range(20):
            eng.run(xs[i % 4], out=outs[i % 4], **kw)
        eng.join(st)
        torch.cuda.synchronize()
        calls = []
        t0 = time.perf_counter()
        for i in range(a.rounds):
            c0 = time.perf_counter()
            eng.run(xs[i % 4], out=outs[i % 4], **kw)
            calls.append(time.perf_counter() - c0)
        eng.join(st)
        torch.cuda.synchronize()
        period = (time.perf_counter() - t0) / a.rounds
        c = sorted(calls)
        print(f"{mode:6s} period {period * 1e6:7.1f} us   host call median {statistics.median(c) * 1e6:6.1f} us  "
              f"p10 {c[len(c) // 10] * 1e6:6.1f}  p90 {c[9 * len(c) // 10] * 1e6:6.1f}", flush=True)
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
