#!/usr/bin/env python3
"""Rehearse the product's C++ round (libomr_dist.so over RCCL) on the GPUs this box has: spawn `world` ranks with
backend "nccl", mapping rank r to device r % device_count, run CppSparseAllreduce rounds in the sync, async and
defer pipelines and check every rank's result against the oracle bit-exactly.
(Several ranks per device only works if RCCL accepts it; on an 8-GPU node every rank gets its own GPU.)"""
import argparse
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "omnireduce-rdma-demo_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def worker(rank, world, port, n, B, density, rounds):
    import oracle
    from omr import Layout
    from omr import cdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", rank % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    L = Layout(n=n, block_size=B)
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B, mode=1, seed=w + 1) for w in range(world)]
    x = torch.from_numpy(bufs[rank].copy()).to(dev)
    out = x.clone()
    eng = cdist.CppSparseAllreduce(L, dev)
    uf = oracle.union_flags([oracle.flags_from_data(b, B) for b in bufs])
    exp = bufs[rank].copy()
    oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, exp)
    ok = True
    for pipe in ("sync", "async", "defer"):
        out.copy_(x)
        for _ in range(rounds):
            eng.run(x, out=out, async_=pipe != "sync", defer=pipe == "defer")
        eng.join()
        torch.cuda.synchronize()
        good = bool((out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all())
        print(f"rank {rank} {pipe}: {'OK' if good else 'MISMATCH'}", flush=True)
        ok &= good
    eng.close()
    dist.barrier()
    dist.destroy_process_group()
    if not ok:
        sys.exit(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--n", type=int, default=4 << 20)
    ap.add_argument("--block-size", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.095)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(worker, args=(a.world, port, a.n, a.block_size, a.density, a.rounds), nprocs=a.world, join=True)


if __name__ == "__main__":
    main()
