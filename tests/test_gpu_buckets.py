"""omr_sparse_buckets_f32: a whole gradient reduced bucket by bucket by the C++ multi-rank round, from device memory
or from PINNED HOST memory (BASELINE config 5's end-to-end path: the reference's registered region res->buf,
common.cc:873-914, filled by the worker, client.cc:401-421, results back in place, client.cc:89), staged through
device buckets with H2D / scan / exchange / D2H overlapped.  Ranks: loopback threads (world 2, 4, 8 on one GPU) and
separate processes over HIP IPC.  Inputs: the reference generator, seeds 1..world, 0.01f fill; every block is
checked against ka[count] (k-fold fp32 sum of 0.01f from +0.0f, server.cc:97-98, :148-150)."""
import ctypes
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

from omr import Layout, cdist, ops

from test_gpu_fullsize import ka_table

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
AR, RS = 0, 1


def rank_input(r, total_n, L, density, dev):
    """Rank r's whole gradient: bucket k is the generator's tensor for worker r + 100 k (a different bitmap per
    bucket), 0.01f blocks."""
    nb_total = total_n // L.block_size
    bms = [ops.gen_bitmap(r + 100 * k, density, L.nb) for k in range(total_n // L.n)]
    bm = np.concatenate(bms)
    x = ops.fill_blocks(torch.from_numpy(bm).to(dev), Layout(n=total_n, block_size=L.block_size))
    assert bm.size == nb_total
    return x, bm


def check(outs, bms, L, world, mode, dev):
    counts = np.sum(bms, axis=0)
    ka = torch.from_numpy(ka_table(world)[counts]).to(dev)
    nbk = L.nb  # blocks per bucket
    bounds = [s * L.rows // world for s in range(world + 1)]
    for r in range(world):
        got = outs[r].to(dev).view(-1, L.block_size)
        exp = ka[:, None].expand(-1, L.block_size)
        if mode == RS:  # the sums land in rank r's shard rows of every bucket; elsewhere its own input
            row_in_bucket = (torch.arange(got.shape[0], device=dev) % nbk) // L.num_lanes
            mine = (row_in_bucket >= bounds[r]) & (row_in_bucket < bounds[r + 1])
            own = torch.from_numpy(bms[r]).to(dev).float()[:, None] * torch.tensor(0.01, device=dev)
            exp = torch.where(mine[:, None], exp, own.expand(-1, L.block_size))
        bad = (got.contiguous().view(torch.int32) != exp.contiguous().view(torch.int32)).any(dim=1)
        if bool(bad.any()):
            idx = torch.nonzero(bad).flatten()
            first = idx[:5].tolist()
            pytest.fail(f"rank {r}: {idx.numel()} of {bad.numel()} blocks differ (bucket of the first: "
                        f"{first[0] // nbk}); first blocks {first}: got {got[idx[:5], 0].tolist()} expected "
                        f"{exp[idx[:5], 0].tolist()} counts {counts[first].tolist()}")


@pytest.mark.parametrize("world,mode,host,bucket_mib,total_mib", [
    (2, AR, True, 16, 64),
    (4, RS, True, 16, 64),
    (2, RS, True, 64, 256),
    (4, AR, True, 64, 256),
    (8, AR, True, 64, 256),   # config-5 shape per rank at 256 MiB: 8 ranks, pinned host, 4 buckets
    (2, AR, True, 256, 4096),  # config 5 per rank (4 GiB pinned host, -r 0.49) in bench's 256 MiB buckets
    (8, RS, True, 64, 256),
    (3, AR, False, 8, 24),    # device memory: deferred rounds only
])
def test_buckets_loopback(gpu, world, mode, host, bucket_mib, total_mib):
    L = Layout.from_bytes(bucket_mib << 20, 256)
    total_n = (total_mib << 20) // 4
    density = 0.49
    D = cdist.load()
    board = D.omr_local_board_create(world)
    bufs, bms = [], []
    for r in range(world):
        x, bm = rank_input(r, total_n, L, density, gpu)
        bms.append(bm)
        bufs.append(x.cpu().pin_memory() if host else x)
    torch.cuda.synchronize()
    errs = []

    def rank(r):
        try:
            torch.cuda.set_device(0)
            d, plan = ctypes.c_void_p(), ctypes.c_void_p()
            assert D.omr_dist_create_local(board, r, ctypes.byref(d)) == 0
            assert D.omr_ar_plan_create(d, L.n, 256, L.num_lanes, 8, ctypes.byref(plan)) == 0
            st = torch.cuda.Stream()
            sent, uni = ctypes.c_uint64(), ctypes.c_uint64()
            rc = D.omr_sparse_buckets_f32(plan, bufs[r].data_ptr(), total_n, mode, ctypes.byref(sent),
                                          ctypes.byref(uni), st.cuda_stream)
            assert rc == 0, D.omr_dist_last_error()
            st.synchronize()
            assert uni.value > 0
            D.omr_ar_plan_destroy(plan)
            D.omr_dist_destroy(d)
        except BaseException as e:  # noqa: BLE001
            errs.append(f"rank {r}: {e!r}")

    th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in th), "a rank is still running after 240 s"
    D.omr_local_board_destroy(board)
    assert not errs, errs
    check(bufs, bms, L, world, mode, gpu)


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", [AR, RS])
def test_buckets_config5_full_shape(gpu, mode):
    """BASELINE config 5 at its own shape: 8 ranks, each with a 4 GiB fp32 gradient in PINNED
    HOST memory (the reference's registered region res->buf, common.cc:873-914, filled by the generator at -r 0.49,
    client.cc:396-421), reduced in place in 256 MiB buckets (16 rounds per rank through the four-buffer staging ring)
    and written back (client.cc:89).  The union of 8 workers at 50 % is about 99.6 %, and 32 of a wave's 64 rows are
    non-zero on average, past the fused pack's LDS stash (the overflow re-read path).  Ranks are loopback threads on
    this GPU (the RCCL form of the same call is tests/test_gpu_rccl_multi.py's world-8 bucket case); every block of
    every rank is checked against ka[count]."""
    import time
    t0 = time.monotonic()
    test_buckets_loopback(gpu, 8, mode, True, 256, 4096)
    print(f"\nconfig 5 full shape, mode {'AR' if mode == AR else 'RS'}: {time.monotonic() - t0:.1f} s wall "
          f"(inputs, 16 buckets x 8 ranks, check)", flush=True)


@pytest.mark.parametrize("world,mode", [(1, AR), (2, AR), (4, RS), (8, AR)])
def test_buckets_loopback_direct(gpu, world, mode, monkeypatch):
    """OMR_BUCKETS_DIRECT=1 (round 6): at N > 1 too, each bucket's round reads and writes the
    mapped pinned bucket in place (the worker scan over PCIe, its pack into device send buffers, the shard sum and the
    unpack storing straight into host memory) instead of the staging ring; N = 1 does so by default."""
    monkeypatch.setenv("OMR_BUCKETS_DIRECT", "1")
    test_buckets_loopback(gpu, world, mode, True, 16, 64)


@pytest.mark.slow
@pytest.mark.timeout(900)
@pytest.mark.parametrize("mode", [AR, RS])
def test_buckets_config5_full_shape_direct(gpu, mode, monkeypatch):
    """Config 5 at its own shape (8 loopback ranks, 4 GiB pinned per rank, 256 MiB buckets, -r 0.49) on the direct
    path: no staging buffer, every rank checked against ka[count]."""
    monkeypatch.setenv("OMR_BUCKETS_DIRECT", "1")
    test_buckets_loopback(gpu, 8, mode, True, 256, 4096)


def test_buckets_one_rank_staging_ring(gpu, monkeypatch):
    """OMR_BUCKETS_STAGED=1: a one-rank group through the four-buffer staging ring instead of its direct launches."""
    monkeypatch.setenv("OMR_BUCKETS_STAGED", "1")
    test_buckets_loopback(gpu, 1, AR, True, 16, 64)


@pytest.mark.parametrize("world,mode", [(2, AR), (4, RS)])
def test_buckets_loopback_staged_writeback(gpu, world, mode, monkeypatch):
    """The previous write-back (each bucket, or the rank's shard, copied back whole from its staging buffer), kept
    behind OMR_BUCKETS_STAGED_D2H for buffers without a device mapping."""
    monkeypatch.setenv("OMR_BUCKETS_STAGED_D2H", "1")
    test_buckets_loopback(gpu, world, mode, True, 16, 64)


@pytest.mark.parametrize("world,mode", [(2, AR), (3, RS)])
def test_buckets_loopback_scan_from_host(gpu, world, mode, monkeypatch):
    """OMR_BUCKETS_SCAN_HOST: the worker scan reads each bucket from the pinned buffer over PCIe and writes its
    non-zero blocks into the staging buffer the rest of the round reads (no H2D copy)."""
    monkeypatch.setenv("OMR_BUCKETS_SCAN_HOST", "1")
    test_buckets_loopback(gpu, world, mode, True, 16, 64)


def test_buckets_reject_pageable(gpu):
    L = Layout.from_bytes(4 << 20, 256)
    D = cdist.load()
    board = D.omr_local_board_create(1)
    d, plan = ctypes.c_void_p(), ctypes.c_void_p()
    assert D.omr_dist_create_local(board, 0, ctypes.byref(d)) == 0
    assert D.omr_ar_plan_create(d, L.n, 256, L.num_lanes, 8, ctypes.byref(plan)) == 0
    pageable = np.zeros(L.n, dtype=np.float32)
    rc = D.omr_sparse_buckets_f32(plan, pageable.ctypes.data, L.n, 0, None, None, None)
    assert rc != 0 and b"pinned" in D.omr_dist_last_error()
    assert D.omr_sparse_buckets_f32(plan, pageable.ctypes.data, L.n + 1, 0, None, None, None) != 0
    D.omr_ar_plan_destroy(plan)
    D.omr_dist_destroy(d)
    D.omr_local_board_destroy(board)


WORKER = os.path.join(HERE, "ipc_bucket_worker.py")


@pytest.mark.parametrize("world,mode", [(2, AR), (3, RS)])
def test_buckets_processes_host(gpu, tmp_path, world, mode):
    """Separate processes (HIP IPC transport), each with its gradient in its own pinned host memory."""
    bucket_mib, total_mib = 8, 32
    uid = cdist.ipc_unique_id().hex()
    procs = []
    for r in range(world):
        cmd = [sys.executable, WORKER, "--rank", str(r), "--world", str(world), "--uid", uid, "--mode", str(mode),
               "--bucket-mib", str(bucket_mib), "--total-mib", str(total_mib), "--out", str(tmp_path / f"r{r}.npy")]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("an IPC rank hung")
    for r, p in enumerate(procs):
        assert p.returncode == 0, logs[r]
    L = Layout.from_bytes(bucket_mib << 20, 256)
    total_n = (total_mib << 20) // 4
    bms = [rank_input(r, total_n, L, 0.49, gpu)[1] for r in range(world)]
    outs = [torch.from_numpy(np.load(tmp_path / f"r{r}.npy")) for r in range(world)]
    check(outs, bms, L, world, mode, gpu)
