"""One rank of the product's C++ round (libomr_dist.so) in its own process: over the HIP-IPC transport, launched by
tests/test_gpu_ipc.py (several of these share the one GPU), or over RCCL under torch.distributed.run, one rank per
GPU (tests/test_gpu_rccl_multi.py, on nodes with enough GPUs).  Writes this rank's outputs to an .npz file."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "omnireduce-rdma-demo_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402  (the generator's inputs only; the round itself runs in libomr_dist.so)
from omr import Layout, cdist, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", choices=("ipc", "rccl"), default="ipc",
                    help="rccl: rank, world and the GPU from torch.distributed.run's environment")
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--world", type=int, default=-1)
    ap.add_argument("--uid", default="", help="hex of the board id (ipc)")
    ap.add_argument("--n", "--floats", dest="n", type=int, required=True)  # --floats under torch.distributed.run
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--density", type=float, default=0.1)
    ap.add_argument("--mode", type=int, default=0, help="OMR_ROUND_* (0 all-reduce, 1 reduce-scatter, 2 dense)")
    ap.add_argument("--pipe", choices=("sync", "async", "defer", "thread", "thread-async"), default="sync",
                    help="thread: deferred rounds issued by the plan's progress thread; thread-async: not deferred")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cycle", type=int, default=0,
                    help="round r runs input (and output buffer) r mod cycle (0: one of each per round); a long run "
                         "thus reuses its buffers as a training loop does")
    ap.add_argument("--workers", type=int, default=0, help="ranks >= this are dedicated aggregators (0: all workers)")
    ap.add_argument("--replan", action="store_true",
                    help="run the rounds, destroy the plan, make a new one on the same transport and run them again "
                         "(the saved outputs are the second plan's)")
    ap.add_argument("--replan-first-n", type=int, default=0,
                    help="--replan: the first plan (and its rounds) at this larger n; the second plan, at --n, then "
                         "reuses the first one's parked, larger exported buffers (ADVICE r04)")
    ap.add_argument("--timeout-ms", type=int, default=0, help="the transport's deadline (omr_dist_set_timeout)")
    ap.add_argument("--fault-rank", type=int, default=-1, help="this rank's first exchange fails (omr_dist_inject_fault)")
    ap.add_argument("--fault-after", type=int, default=0)
    ap.add_argument("--status", default="", help="fault runs: write {error, seconds_to_error} here; exit 3 on an error")
    ap.add_argument("--stall-ms", type=int, default=0,
                    help="queue a busy kernel of about this long on the round's stream before the rounds (a peer that "
                         "falls silent with its part of the exchange still queued)")
    ap.add_argument("--drain", action="store_true", help="fault runs: synchronise the device before leaving")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    stall_per_ms = 0.0
    if a.stall_ms:  # the busy kernel's clock, measured before the group meets (the rounds run under a short deadline)
        torch.cuda.set_device(0)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(10 ** 6)
        s0.record()
        torch.cuda._sleep(10 ** 7)
        s1.record()
        s1.synchronize()
        stall_per_ms = 10 ** 7 / s0.elapsed_time(s1)
    L = Layout(n=a.n, block_size=a.block)
    L0 = Layout(n=a.replan_first_n, block_size=a.block) if a.replan and a.replan_first_n else L
    if a.transport == "rccl":
        a.rank, a.world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        torch.distributed.init_process_group("nccl", device_id=dev)
        nw = a.workers or a.world
        eng = cdist.CppSparseAllreduce(L0, dev, num_workers=nw)
        a.out = a.out.replace("RANK", str(a.rank))
    else:
        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        nw = a.workers or a.world
        eng = cdist.CppSparseAllreduce(L0, dev, transport="ipc", uid=bytes.fromhex(a.uid), rank=a.rank, world=a.world,
                                       num_workers=nw)
    worker = a.rank < nw
    if a.timeout_ms:
        eng.set_timeout(a.timeout_ms)
    if a.fault_rank == a.rank:
        eng.inject_fault(a.fault_after)
    # a different input per round (seed = rank, round): the pipelined rounds must not mix their buffers
    K = a.cycle or a.rounds
    xs, outs = [], []
    for r in range(K):
        if worker:
            x = oracle.fill(oracle.gen_bitmap(a.rank + 10 * r, a.density, L.nb), a.block, mode=1,
                            seed=a.rank + 7 + 31 * r)
            xs.append(torch.from_numpy(x).to(dev))
            outs.append(xs[-1].clone())
        else:  # a dedicated aggregator holds no tensor
            xs.append(None)
            outs.append(None)
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    unx = torch.empty(L.nb, dtype=torch.int32, device=dev)
    sums = {}
    if a.replan:
        if L0 is not L:  # the first plan's rounds on inputs of its own, larger size
            x0 = [torch.from_numpy(oracle.fill(oracle.gen_bitmap(a.rank + 50 + r, a.density, L0.nb), a.block, mode=1,
                                               seed=a.rank + 3 * r)).to(dev) if worker else None for r in range(2)]
            o0 = [x.clone() if x is not None else None for x in x0]
            f0 = torch.zeros(L0.nb, dtype=torch.int32, device=dev)
            n0 = torch.zeros(L0.nb, dtype=torch.int32, device=dev)
            for r in range(a.rounds):
                eng.run(x0[r % 2], out=o0[r % 2], flags=f0, next_offsets=n0, mode=a.mode, async_=a.pipe != "sync",
                        defer=a.pipe in ("defer", "thread"), thread=a.pipe.startswith("thread"))
        else:
            for r in range(a.rounds):
                eng.run(xs[r % K], out=outs[r % K], flags=flags, next_offsets=nxt, union_next=unx, mode=a.mode,
                        async_=a.pipe != "sync", defer=a.pipe in ("defer", "thread"), thread=a.pipe.startswith("thread"))
        eng.join()
        torch.cuda.synchronize()
        eng.replan(L)
        for r in range(K):
            if outs[r] is not None:
                outs[r].copy_(xs[r])
        flags.zero_()
        nxt.zero_()
        unx.zero_()
    if a.stall_ms:
        torch.cuda._sleep(int(stall_per_ms * a.stall_ms))
    t0 = time.monotonic()
    try:
        for r in range(a.rounds):
            eng.run(xs[r % K], out=outs[r % K], flags=flags, next_offsets=nxt, union_next=unx, mode=a.mode,
                    async_=a.pipe != "sync", defer=a.pipe in ("defer", "thread"), thread=a.pipe.startswith("thread"))
            if not worker and a.pipe == "sync":  # a dedicated aggregator's shard sums of this round
                torch.cuda.synchronize()
                sh, r0, r1, ptr, nb = eng.shard()
                t = (torch.as_tensor(ops._DeviceView(ptr, (nb * a.block,), "<f4"), device=dev).clone() if nb
                     else torch.empty(0, device=dev))
                sums[f"sums{r}"] = t.cpu().numpy()
                sums["shard"] = np.array([sh, r0, r1])
        eng.wait()  # (bounded by the transport's deadline: a stuck peer is an error, not a hang)
    except cdist._lib.OmrError as e:
        if not a.status:
            raise
        # a failed round: report, abort (the peers' waits on this rank end at once), leave without the collective
        # clean-up a dead group cannot do
        took = time.monotonic() - t0
        eng.abort()
        c0 = time.monotonic()
        rcs = eng.close()  # (bounded by the deadline even while the device still waits on a peer)
        closed = time.monotonic() - c0
        with open(a.status, "w") as f:
            json.dump({"error": str(e), "seconds_to_error": took, "close_seconds": closed, "close_rcs": list(rcs)}, f)
        print(f"rank {a.rank} failed after {took:.2f} s: {e}; closed in {closed:.2f} s {rcs}", flush=True)
        if a.drain:
            torch.cuda.synchronize()
        os._exit(3)
    torch.cuda.synchronize()
    if a.status:
        with open(a.status, "w") as f:
            json.dump({"error": "", "seconds_to_error": None}, f)
    arrs = dict(flags=flags.cpu().numpy(), next=nxt.cpu().numpy().view(np.uint32),
                unext=unx.cpu().numpy().view(np.uint32), **sums)
    if worker:
        arrs.update({f"out{r}": outs[r].cpu().numpy() for r in range(K)})
    np.savez(a.out, **arrs)
    eng.close()
    if a.transport == "rccl":
        torch.distributed.destroy_process_group()
    print(f"rank {a.rank} ok", flush=True)


if __name__ == "__main__":
    main()
