"""Per-partition single-pass entry point (omr_scan_partition_f32) against the oracle: the reference's per-thread
seam, one host thread per partition (client.cc:384-392 starts NUM_THREADS pthreads, each walking its own
DATA_SIZE_PER_THREAD slice: client.cc:19-31, :168-223), each thread on its own HIP stream, all at once."""
import threading

import numpy as np
import pytest
import torch

import oracle
from omr import Layout, ops

pytestmark = pytest.mark.gpu


def run_threads(x, L, out, flags, nxt, ws, parts=None):
    """Every partition from its own host thread and stream; returns when all are through."""
    parts = list(range(L.num_threads)) if parts is None else parts
    errs = []
    barrier = threading.Barrier(len(parts))

    def worker(t):
        try:
            torch.cuda.set_device(x.device)
            st = torch.cuda.Stream(device=x.device)
            barrier.wait()  # issue together: the calls overlap on the device
            ops.scan_partition(x, L, t, flags, nxt, out, ws, stream=st)
            st.synchronize()
        except BaseException as e:  # noqa: BLE001
            errs.append(f"part {t}: {e!r}")

    th = [threading.Thread(target=worker, args=(t,)) for t in parts]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs


@pytest.mark.parametrize("B,density,mib", [(256, 0.095, 16), (1024, 0.0099, 16), (512, 0.3, 8), (256, 0.0, 4)])
def test_partition_threads_vs_oracle(gpu, B, density, mib):
    L = Layout.from_bytes(mib << 20, B)
    x_np = oracle.fill(oracle.gen_bitmap(3, density, L.nb), B, mode=1, seed=5)
    x = torch.from_numpy(x_np).to(gpu)
    out = torch.full((L.n,), -7.0, device=gpu)  # untouched blocks keep this
    flags = torch.full((L.nb,), -1, dtype=torch.int32, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    ws = ops.scan_workspace(L, device=gpu)
    run_threads(x, L, out, flags, nxt, ws)
    f = oracle.flags_from_data(x_np, B)
    assert (flags.cpu().numpy() == f).all()
    assert (nxt.cpu().numpy().view(np.uint32) == oracle.next_offsets(f, L.n, B, L.num_lanes, L.num_threads)).all()
    exp = np.full(L.n, -7.0, dtype=np.float32)
    oracle.block_sum([x_np], L.n, B, L.num_lanes, L.num_threads, f, exp)
    assert (out.cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all()
    assert (ws.cpu().numpy() == 0).all(), "workspace left zeroed"


def test_partition_subset_leaves_others_untouched(gpu):
    L = Layout.from_bytes(8 << 20, 256)
    x_np = oracle.fill(oracle.gen_bitmap(1, 0.2, L.nb), 256)
    x = torch.from_numpy(x_np).to(gpu)
    out = torch.full((L.n,), -7.0, device=gpu)
    flags = torch.full((L.nb,), -1, dtype=torch.int32, device=gpu)
    nxt = torch.full((L.nb,), 5, dtype=torch.int32, device=gpu)
    ws = ops.scan_workspace(L, device=gpu)
    run_threads(x, L, out, flags, nxt, ws, parts=[2, 5])
    f = oracle.flags_from_data(x_np, 256)
    full_next = oracle.next_offsets(f, L.n, 256, L.num_lanes, L.num_threads)
    per = L.nb // L.num_threads
    gf, gn = flags.cpu().numpy(), nxt.cpu().numpy().view(np.uint32)
    for t in range(L.num_threads):
        sl = slice(t * per, (t + 1) * per)
        if t in (2, 5):
            assert (gf[sl] == f[sl]).all() and (gn[sl] == full_next[sl]).all()
        else:
            assert (gf[sl] == -1).all() and (gn[sl] == 5).all()


def test_partition_bad_index(gpu):
    L = Layout.from_bytes(4 << 20, 256)
    x = torch.zeros(L.n, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    with pytest.raises(Exception, match="out of range"):
        ops.scan_partition(x, L, L.num_threads, None, nxt, None, ops.scan_workspace(L, device=gpu))


@pytest.mark.slow
def test_partition_threads_config2(gpu):
    """Config 2 (256 MiB, B=256, -r 0.095) through 8 concurrent per-partition calls == the whole-tensor kernel
    == the generator bitmap (size-independent properties; no CPU pass over 256 MiB)."""
    L = Layout.from_bytes(256 << 20, 256)
    bm = ops.gen_bitmap(0, 0.095, L.nb)
    x = ops.fill_blocks(torch.from_numpy(bm).to(gpu), L)
    out = torch.zeros(L.n, device=gpu)
    flags = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    nxt = torch.zeros(L.nb, dtype=torch.int32, device=gpu)
    run_threads(x, L, out, flags, nxt, ops.scan_workspace(L, device=gpu))
    ref = ops.ScanSumPlan(L, 1, device=gpu, fused=True)
    ref_out = torch.zeros(L.n, device=gpu)
    r = ref.run([x], ref_out)
    torch.cuda.synchronize()
    assert (flags.cpu().numpy() == bm).all()
    assert torch.equal(nxt, r.next_offsets[0])
    assert torch.equal(out.view(torch.int32), ref_out.view(torch.int32))
