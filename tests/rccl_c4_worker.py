"""One rank of BASELINE config 4 (or config 5's bucketed path) over RCCL, one process per GPU under
torch.distributed.run (tests/test_gpu_rccl_multi.py; needs a node with `world` GPUs).

c4:      each rank is worker r with its own 256 MiB tensor (generator seed r+1, -r 0.095, the reference's 0.01f fill:
         client.cc:396-421) and the aggregator of shard r; deferred rounds in reduce-scatter and all-reduce mode.
buckets: omr_sparse_buckets_f32 on the rank's gradient in PINNED HOST memory, bucket k = the generator's tensor for
         worker r + 100 k at -r 0.49 (config 5's end-to-end path).
Checked on the device (no CPU pass over the data): every summed block == ka[count] (the k-fold fp32 sum of 0.01f from
+0.0f, server.cc:97-98, :148-150: the reference CHECK's known answer, client.cc:449-465), blocks outside the rank's
part untouched, flags == the bitmap, the worker's and the aggregator's next chains == the oracle's (client.cc:19-31,
server.cc:86-96).  Rank r writes "ok" (or the failure) to --out with RANK replaced."""
import argparse
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "omnireduce-rdma-demo_amd"), os.path.join(ROOT, "oracle"), HERE):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402  (checker: bitmaps and next chains)
from omr import Layout, cdist, ops  # noqa: E402
from test_gpu_fullsize import ka_table  # noqa: E402

AR, RS = 0, 1


def check_c4(eng, L, rank, world, rounds, dev):
    bms = [ops.gen_bitmap(w, 0.095, L.nb) for w in range(world)]
    counts = np.sum(bms, axis=0).astype(np.int64)
    union = (counts > 0).astype(np.int32)
    ka = torch.from_numpy(ka_table(world)[counts]).to(dev)
    bounds = [s * L.rows // world for s in range(world + 1)]
    x = ops.fill_blocks(torch.from_numpy(bms[rank]).to(dev), L)
    own = x.clone()
    flags = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    unx = torch.zeros(L.nb, dtype=torch.int32, device=dev)
    row = torch.arange(L.nb, device=dev) // L.num_lanes
    mine = (row >= bounds[rank]) & (row < bounds[rank + 1])
    for mode in (RS, AR):
        outs = [x.clone() for _ in range(3)]
        for k in range(rounds):
            eng.run(x, out=outs[k % 3], flags=flags, next_offsets=nxt, union_next=unx, mode=mode, async_=True,
                    defer=True)
        eng.wait()  # bounded by the transport's deadline (a stuck peer is an error, not a hang)
        for out in outs[:min(rounds, 3)]:
            got = out.view(L.nb, L.block_size).view(torch.int32)
            exp = ka[:, None].expand(-1, L.block_size)
            if mode == RS:
                exp = torch.where(mine[:, None], exp, own.view(L.nb, L.block_size))
            assert torch.equal(got, exp.contiguous().view(torch.int32)), f"mode {mode}: sums differ from ka[count]"
        assert torch.equal(x, own), "x was written"
        assert (flags.cpu().numpy() == bms[rank]).all(), "flags"
        assert (nxt.cpu().numpy().view(np.uint32) ==
                oracle.next_offsets(bms[rank], L.n, L.block_size, L.num_lanes, 8)).all(), "worker next chain"
        assert (unx.cpu().numpy().view(np.uint32) ==
                oracle.next_offsets(union, L.n, L.block_size, L.num_lanes, 8)).all(), "aggregator chain"


def check_buckets(eng, L, rank, world, total_mib, dev):
    from test_gpu_buckets import rank_input
    total_n = (total_mib << 20) // 4
    bms_all = []
    for r in range(world):
        bms_all.append(np.concatenate([ops.gen_bitmap(r + 100 * k, 0.49, L.nb) for k in range(total_n // L.n)]))
    x, bm = rank_input(rank, total_n, L, 0.49, dev)
    counts = np.sum(bms_all, axis=0)
    ka = torch.from_numpy(ka_table(world)[counts]).to(dev)
    bounds = [s * L.rows // world for s in range(world + 1)]
    for mode in (AR, RS):
        host = x.cpu().pin_memory()
        eng.run_buckets(host, mode=mode)
        got = host.to(dev).view(-1, L.block_size)
        exp = ka[:, None].expand(-1, L.block_size)
        if mode == RS:
            rib = (torch.arange(got.shape[0], device=dev) % L.nb) // L.num_lanes
            mine = (rib >= bounds[rank]) & (rib < bounds[rank + 1])
            exp = torch.where(mine[:, None], exp, x.view(-1, L.block_size))
        assert torch.equal(got.contiguous().view(torch.int32), exp.contiguous().view(torch.int32)), \
            f"buckets mode {mode}: blocks differ"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", choices=("c4", "buckets"), required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--total-mib", type=int, default=1024)
    ap.add_argument("--fault-rank", type=int, default=-1,
                    help="this rank's first exchange fails (omr_dist_inject_fault): the run must end at once, with "
                         "the rank's error in its --out file and a non-zero exit, instead of hanging its peers")
    ap.add_argument("--fault-op", choices=("exchange", "allgather"), default="exchange",
                    help="which transport operation fails (at world 1 a round has no exchange: use allgather)")
    ap.add_argument("--timeout-ms", type=int, default=0, help="the transport's deadline (default 60 s)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.distributed.init_process_group("nccl", device_id=dev)
    L = Layout.from_bytes(256 << 20, 256)
    eng = cdist.CppSparseAllreduce(L, dev)
    if a.timeout_ms:
        eng.set_timeout(a.timeout_ms)
    if a.fault_rank == rank:
        if world == 1:  # a one-rank group's round is its scan alone: run the multi-rank round's path to reach the op
            eng.test_world1_round(True)
        eng.inject_fault(0) if a.fault_op == "exchange" else eng.inject_allgather_fault()
    out = a.out.replace("RANK", str(rank))
    t0 = time.monotonic()
    try:
        if a.case == "c4":
            check_c4(eng, L, rank, world, a.rounds, dev)
        else:
            check_buckets(eng, L, rank, world, a.total_mib, dev)
    except Exception:  # noqa: BLE001
        # fail fast: report, abort the transport (RCCL's communicators; the peers end at their deadlines or when the
        # launcher stops them on this exit), and leave without the collective clean-up a broken group cannot do
        msg = traceback.format_exc()
        with open(out, "w") as f:
            f.write(f"rank {rank} failed after {time.monotonic() - t0:.2f} s\n{msg}")
        print(f"rank {rank} FAILED after {time.monotonic() - t0:.2f} s: {msg.splitlines()[-1]}", file=sys.stderr,
              flush=True)
        eng.abort()
        os._exit(1)
    eng.close()
    torch.distributed.destroy_process_group()
    with open(out, "w") as f:
        f.write("ok")
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
