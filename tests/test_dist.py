"""Multi-rank sparse all-reduce — the N>1 protocol on world_size 2..5 over gloo.

CPU tests run the protocol of the product's C++ round (csrc/omr_dist.hip) through its Python twin
tests/dist_twin.py (roles, shard bounds, mask all-gather, packed-stream
offsets, grouped send/recv, in-place scatter) with the oracle-backed CpuBackend; the gpu test runs the same
protocol with the HIP kernels (HipBackend) on one GPU shared by two processes, host-staged gloo comms.
Expected result = the reference's in-place allreduce: every worker's buffer becomes the rank-order sum over
the union of non-zero blocks plus lane heads (client.cc:89, :449-465; server.cc:97-98)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, B, density, mode, use_gpu, errq, round_mode=0, num_workers=0):
    try:
        sys.path[:0] = [HERE, os.path.join(HERE, "..", "oracle"), os.path.join(HERE, "..", "omnireduce-rdma-demo_amd")]
        import oracle
        from cpu_backend import CpuBackend, HostStagedComm
        from omr import Layout
        import dist_twin as odist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        L = Layout(n=n, block_size=B)
        if num_workers:  # m workers + (world - m) dedicated aggregators
            _roles(rank, world, num_workers, L, B, density, mode, round_mode)
            dist.barrier()
            dist.destroy_process_group()
            return
        bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B, mode=mode, seed=w + 1) for w in range(world)]
        if use_gpu:
            dev = torch.device("cuda:0")
            x = torch.from_numpy(bufs[rank].copy()).to(dev)
            eng = odist.SparseAllreduce(L, device=dev, comm=HostStagedComm())
        else:
            x = torch.from_numpy(bufs[rank].copy())
            eng = odist.SparseAllreduce(L, device="cpu", backend=CpuBackend(L, world), comm=odist.TorchComm())
        if round_mode == 1:  # reduce-scatter: own shard of the write set gets the sums, the rest is untouched
            out = x.clone()
            res = eng.run(x, out=out, mode=1)
            if use_gpu:
                torch.cuda.synchronize()
            flags = [oracle.flags_from_data(b, B) for b in bufs]
            uf = oracle.union_flags(flags)
            full = bufs[rank].copy()
            oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, full)
            r0, r1 = eng.bounds[rank], eng.bounds[rank + 1]
            exp = bufs[rank].copy()
            lo, hi = r0 * L.num_lanes * B, r1 * L.num_lanes * B
            exp[lo:hi] = full[lo:hi]
            got = out.cpu().numpy()
            assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"rank {rank}: reduce-scatter mismatch"
            dist.barrier()
            dist.destroy_process_group()
            return
        for it in range(2):  # second round: results feed the next round's scan (values change, masks do not)
            res = eng.run(x)
            if use_gpu:
                torch.cuda.synchronize()
            flags = [oracle.flags_from_data(b, B) for b in bufs]
            uf = oracle.union_flags(flags)
            exp = bufs[rank].copy()
            oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, exp)
            got = x.cpu().numpy()
            assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"rank {rank} round {it}: sum mismatch"
            assert (res.flags.cpu().numpy() == flags[rank]).all()
            nx = oracle.next_offsets(flags[rank], L.n, B, L.num_lanes, L.num_threads)
            assert (res.next_offsets.cpu().numpy().view(np.uint32) == nx).all(), "worker chain"
            un = oracle.next_offsets(uf, L.n, B, L.num_lanes, L.num_threads)
            assert (res.union_next.cpu().numpy().view(np.uint32) == un).all(), "aggregator chain"
            # every worker now holds the allreduced tensor: next round's inputs
            allb = [None] * world
            gathered = [torch.empty(L.n) for _ in range(world)]
            dist.all_gather(gathered, x.cpu())
            bufs = [g.numpy().copy() for g in gathered]
            assert all((b.view(np.uint32) == got.view(np.uint32)).all() for b in bufs)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # report to the parent
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def _roles(rank, world, m, L, B, density, mode, round_mode):
    """Dedicated aggregators: workers 0..m-1 hold tensors, ranks m.. aggregate shard rank - m and hold none."""
    import oracle
    from cpu_backend import CpuBackend
    import dist_twin as odist
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B, mode=mode, seed=w + 1) for w in range(m)]
    eng = odist.SparseAllreduce(L, device="cpu", backend=CpuBackend(L, m), comm=odist.TorchComm(), num_workers=m)
    x = torch.from_numpy(bufs[rank].copy()) if rank < m else None
    out = x.clone() if x is not None else None
    res = eng.run(x, out=out, mode=round_mode)
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    uf = oracle.union_flags(flags)
    full = np.zeros(L.n, dtype=np.float32)
    oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, full)
    assert (res.union_next.numpy().view(np.uint32) ==
            oracle.next_offsets(uf, L.n, B, L.num_lanes, L.num_threads)).all(), "aggregator chain"
    if rank < m:
        exp = bufs[rank].copy()
        if round_mode == 0:
            oracle.block_sum(bufs, L.n, B, L.num_lanes, L.num_threads, uf, exp)
        got = out.numpy()
        assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"worker {rank}"
    else:  # the aggregator's packed shard sums: the write set of its rows in block order (server.cc:143-147)
        j = rank - m
        r0, r1 = eng.bounds[j], eng.bounds[j + 1]
        heads = (np.arange(L.nb) // L.num_lanes) % L.rows_per_part == 0
        blocks = np.arange(r0 * L.num_lanes, r1 * L.num_lanes)
        sel = blocks[(uf.astype(bool) | heads)[r0 * L.num_lanes:r1 * L.num_lanes]]
        exp = full.reshape(L.nb, B)[sel].reshape(-1)
        got = eng.sums[:exp.size].numpy()
        total = int(np.count_nonzero(uf.astype(bool) | heads))
        assert res.union_blocks == (sel.size if round_mode == 1 else total)
        assert (got.view(np.uint32) == exp.view(np.uint32)).all(), f"aggregator {j}"


def _run(world, n, B, density, mode, use_gpu=False, round_mode=0, num_workers=0):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, B, density, mode, use_gpu, errq, round_mode,
                                               num_workers))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("world,B,density,mode", [
    (2, 256, 0.095, 1),
    (2, 1024, 0.0099, 0),
    (3, 256, 0.3, 1),   # shards of unequal row counts
    (4, 512, 0.49, 1),
])
def test_sparse_allreduce_cpu(world, B, density, mode):
    _run(world, 1 << 20, B, density, mode)


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_reduce_scatter_cpu(world):
    _run(world, 1 << 20, 256, 0.3, 1, round_mode=1)


def test_sparse_allreduce_all_zero_cpu():
    _run(2, 1 << 20, 256, 0.0, 0)


@pytest.mark.gpu
def test_sparse_allreduce_gpu_two_procs(gpu):
    _run(2, 4 << 20, 256, 0.095, 1, use_gpu=True)


@pytest.mark.parametrize("world,m,round_mode", [(3, 2, 0), (4, 2, 0), (4, 3, 1), (5, 2, 1)])
def test_dedicated_aggregators_cpu(world, m, round_mode):
    """m workers + world - m dedicated aggregators (the reference's separate servers) over gloo."""
    _run(world, 1 << 20, 256, 0.3, 1, round_mode=round_mode, num_workers=m)
