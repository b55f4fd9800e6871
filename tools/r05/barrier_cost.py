"""The fixed cost of the end of bench's timed region at N>1 (under torch.distributed.run, one rank per GPU, NCCL = RCCL):
K back-to-back launches of the headline kernel, then (A) synchronize, barrier, synchronize -- bench's sequence -- or
(B) barrier, synchronize (the barrier's collective is queued behind the launches on the NCCL stream, which waits for
the current stream), or (C) synchronize only.  Host time per call minus the kernels' span (events), median of 30.
usage: python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/r05/barrier_cost.py"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from omr import Layout, ops, timing  # noqa: E402

local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dev = torch.device("cuda", local)
dist.init_process_group("nccl", device_id=dev)
K = 20
L = Layout.from_bytes(256 << 20, 256)
bm = ops.gen_bitmap(0, 0.095, L.nb)
sets = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0) for _ in range(4)]
plan = ops.ScanSumPlan(L, 1, device=dev, fused=True)
stream = torch.cuda.current_stream(dev)
launches = [plan.bind(x, x, stream) for x in sets]
span = (timing.Event(), timing.Event())
for i in range(10):
    launches[i % 4]()
torch.cuda.synchronize()
dist.barrier()


def one(method):
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    span[0].record(stream)
    for i in range(K):
        launches[i % 4]()
    span[1].record(stream)
    if method == "A":
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
    elif method == "B":
        dist.barrier()
        torch.cuda.synchronize()
    else:
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) * 1e6
    return dt, dt - span[0].elapsed_time(span[1]) * 1e3


res = {m: [] for m in "ABC"}
for _ in range(30):
    for m in "ABC":
        res[m].append(one(m))
if dist.get_rank() == 0:
    for m, v in res.items():
        print(f"{m}: us per {K}-step call median {statistics.median(a for a, _ in v):.1f} | host - kernels' span median "
              f"{statistics.median(b for _, b in v):.1f} min {min(b for _, b in v):.1f}", flush=True)
dist.destroy_process_group()
