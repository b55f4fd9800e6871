"""Device-tensor front end of the C ABI (include/omr.h).

Every function here is a thin call through libomr.so on torch-allocated HBM buffers and the current HIP
stream; torch provides memory and streams only.  Names follow the reference: the worker scan
(client.cc:19-31), the aggregator sum (server.cc:83-99), the generator (client.cc:396-421).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from .layout import MESSAGE_SIZE, NUM_SLOTS, Layout


def _stream(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("expected a device (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t.data_ptr()


def _ptr_array(ts: Sequence[torch.Tensor]):
    arr = (ctypes.c_void_p * len(ts))()
    for i, t in enumerate(ts):
        arr[i] = _ptr(t)
    return arr


def _check_f32(t: torch.Tensor, n: int, name: str) -> None:
    if t.dtype != torch.float32 or t.numel() != n:
        raise ValueError(f"{name}: expected float32[{n}], got {t.dtype}[{t.numel()}]")


# ------------------------------------------------------------------ generator (client.cc:396-421)

def gen_bitmap(worker_id: int, density_ratio: float, num_blocks: int) -> np.ndarray:
    """The reference bitmap of worker `worker_id` (srand(myId+1); rand()%100/(double)101 < r)."""
    lib = _lib.load()
    bm = np.empty(num_blocks, dtype=np.int32)
    cnt = ctypes.c_uint64(0)
    _lib.check(lib.omr_gen_bitmap(worker_id, float(density_ratio), num_blocks,
                                  bm.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cnt)), "omr_gen_bitmap")
    return bm


def fill_blocks(bitmap: torch.Tensor, layout: Layout, mode: int = 0, seed: int = 0,
                out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """Device fill from a device int32 bitmap: mode 0 = 0.01f (client.cc:415-419), 1 = hashed [-1,1)."""
    if bitmap.dtype != torch.int32 or bitmap.numel() != layout.nb:
        raise ValueError("bitmap must be int32[nb]")
    if out is None:
        out = torch.empty(layout.n, dtype=torch.float32, device=bitmap.device)
    _check_f32(out, layout.n, "out")
    _lib.check(_lib.load().omr_fill_blocks_f32(_ptr(bitmap), layout.nb, layout.block_size, mode, seed,
                                               _ptr(out), _stream(stream)), "omr_fill_blocks_f32")
    return out


def make_worker_buffer(worker_id: int, density_ratio: float, layout: Layout, device="cuda", mode: int = 0,
                       seed: Optional[int] = None) -> torch.Tensor:
    bm = torch.from_numpy(gen_bitmap(worker_id, density_ratio, layout.nb)).to(device)
    return fill_blocks(bm, layout, mode=mode, seed=worker_id + 1 if seed is None else seed)


# ------------------------------------------------------------------ scan + sum

@dataclass
class ScanResult:
    flags: Optional[torch.Tensor]  # int32 [m][nb]
    masks: torch.Tensor  # uint64-as-int64 [m(+1)][rows]
    next_offsets: Optional[torch.Tensor]  # uint32-as-int32 [m(+1)][nb]
    out: Optional[torch.Tensor]


class ScanSumPlan:
    """Preallocated outputs for repeated fused scan+sum launches (no allocation per call, capturable).

    flags        int32  [m, nb]             per-worker block flags (the reference's int *bitmap)
    masks        int64  [m(+1), rows]       per-worker row masks (+ the union row at index m when m > 1)
    next_offsets int32  [m(+1), nb]         per-worker next-offset chains (+ the aggregator chain), uint32 bits
    """

    def __init__(self, layout: Layout, m: int = 1, with_flags: bool = True, with_next: bool = True,
                 device="cuda", fused: bool = False, row_masks: bool = False):
        """fused=True (m = 1 only): one single-pass launch (omr_scan_sum_fused_f32) producing flags, next
        offsets and the aggregated blocks; with row_masks=True it is the multi-rank round's worker scan
        (omr_worker_scan_f32), which also ORs the row masks into `masks` (zeroed before each run)."""
        if not 1 <= m <= _lib.OMR_MAX_WORKERS:
            raise ValueError(f"m={m} out of range")
        lib = _lib.load()
        _lib.check(lib.omr_layout_check(layout.n, layout.block_size, layout.num_lanes, layout.num_threads),
                   "omr_layout_check")
        if fused and (m != 1 or not with_next):
            raise ValueError("the fused single-pass kernel is the m = 1 step with next offsets")
        self.layout, self.m, self.fused = layout, m, fused
        arrays = m if m == 1 else m + 1
        self.flags = torch.empty((m, layout.nb), dtype=torch.int32, device=device) if with_flags else None
        self.row_masks = bool(fused and row_masks)
        self.masks = (None if fused and not row_masks else
                      torch.zeros((arrays, layout.rows), dtype=torch.int64, device=device))
        self.next_offsets = (torch.empty((arrays, layout.nb), dtype=torch.int32, device=device)
                             if with_next else None)
        ws = lib.omr_scan_workspace_bytes(layout.n, layout.block_size, layout.num_lanes, layout.num_threads)
        self.workspace = torch.zeros(max(ws, 16), dtype=torch.uint8, device=device) if fused else None

    def bind(self, buf: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None):
        """The fused m = 1 launch with its arguments checked and converted once: returns a zero-argument callable
        that issues omr_scan_sum_fused_f32 (one C call per step, for a host-light loop; raises on error)."""
        if not self.fused or self.row_masks or self.m != 1:
            raise ValueError("bind(): the fused m = 1 scan + sum only")
        L = self.layout
        _check_f32(buf, L.n, "buf")
        if out is not None:
            _check_f32(out, L.n, "out")
        fn = _lib.load().omr_scan_sum_fused_f32
        args = (_ptr(buf), L.n, L.block_size, L.num_lanes, L.num_threads, _ptr(self.flags), _ptr(self.next_offsets),
                _ptr(out), _ptr(self.workspace), self.workspace.numel(), _stream(stream))

        def launch():
            rc = fn(*args)
            if rc:
                _lib.check(rc, "omr_scan_sum_fused_f32")
        return launch

    def run(self, bufs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None, stream=None,
            with_next: bool = True, zero_masks: bool = True) -> ScanResult:
        """Fused scan (+ sum into `out`) and, unless with_next=False, the next-offset chains."""
        L = self.layout
        if len(bufs) != self.m:
            raise ValueError(f"expected {self.m} worker buffers, got {len(bufs)}")
        for i, b in enumerate(bufs):
            _check_f32(b, L.n, f"bufs[{i}]")
        if out is not None:
            _check_f32(out, L.n, "out")
        if self.fused and self.row_masks:
            if zero_masks:
                self.masks.zero_()
            _lib.check(_lib.load().omr_worker_scan_f32(
                _ptr(bufs[0]), L.n, L.block_size, L.num_lanes, L.num_threads, _ptr(self.flags),
                _ptr(self.next_offsets), _ptr(self.masks), _ptr(out), _ptr(self.workspace), self.workspace.numel(),
                _stream(stream)), "omr_worker_scan_f32")
            return ScanResult(self.flags, self.masks, self.next_offsets, out)
        if self.fused:
            _lib.check(_lib.load().omr_scan_sum_fused_f32(
                _ptr(bufs[0]), L.n, L.block_size, L.num_lanes, L.num_threads, _ptr(self.flags),
                _ptr(self.next_offsets), _ptr(out), _ptr(self.workspace), self.workspace.numel(), _stream(stream)),
                "omr_scan_sum_fused_f32")
            return ScanResult(self.flags, self.masks, self.next_offsets, out)
        arr = _ptr_array(bufs)
        nxt = self.next_offsets if with_next else None
        _lib.check(_lib.load().omr_scan_sum_f32(arr, self.m, L.n, L.block_size, L.num_lanes, L.num_threads,
                                                _ptr(self.flags), _ptr(self.masks), _ptr(nxt),
                                                _ptr(out), _stream(stream)), "omr_scan_sum_f32")
        return ScanResult(self.flags, self.masks, self.next_offsets, out)

    def resolve_next(self, stream=None) -> torch.Tensor:
        """Next-offset chains from the masks of the last run (the second kernel of run())."""
        L = self.layout
        if self.next_offsets is None:
            raise ValueError("plan built with with_next=False")
        _lib.check(_lib.load().omr_next_offsets(_ptr(self.masks), self.masks.shape[0], L.n, L.block_size,
                                                L.num_lanes, L.num_threads, _ptr(self.next_offsets),
                                                _stream(stream)), "omr_next_offsets")
        return self.next_offsets


def scan_workspace(layout: Layout, device="cuda") -> torch.Tensor:
    """Zeroed workspace for the single-pass kernels (omr_scan_workspace_bytes; one per concurrently running whole-
    tensor call, or ONE shared by concurrent per-partition calls)."""
    ws = _lib.load().omr_scan_workspace_bytes(layout.n, layout.block_size, layout.num_lanes, layout.num_threads)
    return torch.zeros(max(ws, 16), dtype=torch.uint8, device=device)


def scan_partition(buf: torch.Tensor, layout: Layout, part: int, flags: Optional[torch.Tensor],
                   next_offsets: torch.Tensor, out: Optional[torch.Tensor], workspace: torch.Tensor,
                   stream=None) -> None:
    """The single-pass worker step for partition `part` only (omr_scan_partition_f32): the reference's per-thread
    seam, worker thread res->threadId walking its own DATA_SIZE_PER_THREAD slice (client.cc:19-31, :168-223).
    flags / next_offsets / out are whole-tensor arrays (global indexing); only the partition's entries are written.
    Safe to call from several host threads at once, one partition and one stream each (ctypes drops the GIL)."""
    _check_f32(buf, layout.n, "buf")
    if out is not None:
        _check_f32(out, layout.n, "out")
    lib = _lib.load()
    rc = lib.omr_scan_partition_f32(_ptr(buf), layout.n, layout.block_size, layout.num_lanes, layout.num_threads,
                                    part, _ptr(flags), _ptr(next_offsets), _ptr(out), _ptr(workspace),
                                    workspace.numel(), _stream(stream))
    _lib.check(rc, "omr_scan_partition_f32")


def scan(buf: torch.Tensor, layout: Layout, stream=None) -> ScanResult:
    """Worker-side scan (client.cc:19-31): flags, row masks and next offsets of one gradient buffer."""
    return ScanSumPlan(layout, 1, device=buf.device).run([buf], None, stream)


def scan_sum(bufs: Sequence[torch.Tensor], layout: Layout, out: Optional[torch.Tensor] = None,
             stream=None) -> ScanResult:
    """m worker scans + aggregator sum (server.cc:83-99) in one HBM pass."""
    if out is None:
        out = torch.zeros(layout.n, dtype=torch.float32, device=bufs[0].device)
    return ScanSumPlan(layout, len(bufs), device=bufs[0].device).run(bufs, out, stream)


def next_offsets(masks: torch.Tensor, layout: Layout, stream=None) -> torch.Tensor:
    """Next-offset chains from row masks [count, rows] (client.cc:19-31; server.cc:86-96 on a union)."""
    if masks.dim() == 1:
        masks = masks.view(1, -1)
    if masks.dtype != torch.int64 or masks.shape[1] != layout.rows:
        raise ValueError("masks must be int64[count, rows]")
    count = masks.shape[0]
    nxt = torch.empty((count, layout.nb), dtype=torch.int32, device=masks.device)
    _lib.check(_lib.load().omr_next_offsets(_ptr(masks.contiguous()), count, layout.n, layout.block_size,
                                            layout.num_lanes, layout.num_threads, _ptr(nxt), _stream(stream)),
               "omr_next_offsets")
    return nxt


# ------------------------------------------------------------------ compaction and block movement

class CompactPlan:
    def __init__(self, rows: int, num_lanes: int, device="cuda"):
        self.rows, self.num_lanes = rows, num_lanes
        ws = _lib.load().omr_compact_workspace_bytes(rows)
        self.workspace = torch.empty(ws, dtype=torch.uint8, device=device)
        self.count = torch.zeros(1, dtype=torch.int32, device=device)
        self.block_list = torch.empty(rows * num_lanes, dtype=torch.int32, device=device)

    def run(self, masks: torch.Tensor, row_begin: int = 0, row_end: Optional[int] = None, stream=None):
        row_end = self.rows if row_end is None else row_end
        _lib.check(_lib.load().omr_compact(_ptr(masks), row_begin, row_end, self.num_lanes,
                                           _ptr(self.block_list), _ptr(self.count), _ptr(self.workspace),
                                           self.workspace.numel(), _stream(stream)), "omr_compact")
        return self.block_list, self.count


def compact(masks: torch.Tensor, layout: Layout, row_begin: int = 0, row_end: Optional[int] = None,
            stream=None) -> torch.Tensor:
    """Global indices of the non-zero blocks of rows [row_begin, row_end), increasing (synchronises)."""
    plan = CompactPlan(layout.rows, layout.num_lanes, device=masks.device)
    lst, cnt = plan.run(masks.contiguous(), row_begin, row_end, stream)
    return lst[: int(cnt.item())].clone()


def gather_blocks(src: torch.Tensor, block_list: torch.Tensor, num: int, block_size: int,
                  packed: torch.Tensor, stream=None) -> torch.Tensor:
    """Pack listed blocks contiguously (worker gather, common.cc:405-407)."""
    if num:
        _lib.check(_lib.load().omr_gather_blocks_f32(_ptr(src), _ptr(block_list), num, block_size,
                                                     _ptr(packed), _stream(stream)), "omr_gather_blocks_f32")
    return packed


def scatter_blocks(packed: torch.Tensor, block_list: torch.Tensor, num: int, block_size: int,
                   dst: torch.Tensor, stream=None) -> torch.Tensor:
    """Write packed blocks back in place (worker result copy, client.cc:89)."""
    if num:
        _lib.check(_lib.load().omr_scatter_blocks_f32(_ptr(packed), _ptr(block_list), num, block_size,
                                                      _ptr(dst), _stream(stream)), "omr_scatter_blocks_f32")
    return dst


def block_sum(inputs: Sequence[torch.Tensor], block_list: torch.Tensor, num: int, block_size: int,
              out: torch.Tensor, stream=None) -> torch.Tensor:
    """out[b] = ((0 + in_0[b]) + in_1[b]) + ... for listed blocks b (server.cc:97-98, rank order)."""
    if num:
        arr = _ptr_array(inputs)
        _lib.check(_lib.load().omr_block_sum_f32(arr, len(inputs), _ptr(block_list), num, block_size,
                                                 _ptr(out), _stream(stream)), "omr_block_sum_f32")
    return out


# ------------------------------------------------------------------ host-resident end-to-end path

class HostPlan:
    """omr_host_plan: H2D -> in-place scan + aggregate -> D2H over row chunks on three HIP streams, for a
    gradient that starts and ends in pinned host memory (the reference's registered region)."""

    def __init__(self, layout: Layout, chunk_rows: int = 512):
        self.layout = layout
        self._p = ctypes.c_void_p()
        rc = _lib.load().omr_host_plan_create(layout.n, layout.block_size, layout.num_lanes, layout.num_threads,
                                              chunk_rows, ctypes.byref(self._p))
        if rc != 0:
            raise _lib.OmrError(f"omr_host_plan_create rc={rc}: {_lib.load().omr_host_last_error().decode()}")

    def run(self, host_buf: torch.Tensor, flags: Optional[torch.Tensor] = None,
            next_offsets: Optional[torch.Tensor] = None, zero_copy: bool = False) -> float:
        """zero_copy: the single-pass kernel reads and writes the pinned buffer in place over PCIe instead of
        staging it through HBM (omr_host_scan_sum_zero_copy_f32)."""
        L = self.layout
        for t, n, dt in ((host_buf, L.n, torch.float32), (flags, L.nb, torch.int32),
                         (next_offsets, L.nb, torch.int32)):
            if t is not None and (t.is_cuda or t.dtype != dt or t.numel() != n or not t.is_contiguous()):
                raise ValueError("host tensors must be contiguous CPU tensors of the layout's size")
        secs = ctypes.c_double()
        lib = _lib.load()
        fn = lib.omr_host_scan_sum_zero_copy_f32 if zero_copy else lib.omr_host_scan_sum_f32
        rc = fn(self._p, host_buf.data_ptr(), flags.data_ptr() if flags is not None else None,
                next_offsets.data_ptr() if next_offsets is not None else None, ctypes.byref(secs))
        if rc != 0:
            raise _lib.OmrError(f"omr_host_scan_sum{'_zero_copy' if zero_copy else ''}_f32 rc={rc}: "
                                f"{lib.omr_host_last_error().decode()}")
        return secs.value

    def close(self):
        if self._p:
            _lib.load().omr_host_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ message-level round (wire format)

class _DeviceView:
    """A device buffer owned by the library, exposed to torch through __cuda_array_interface__ (no copy)."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (ptr, False),
                                         "version": 3, "strides": None}


class MessageRound:
    """The round as the reference's messages (include/omr.h omr_msg_*): m workers on one device, every worker
    message and aggregator reply in the wire format of common.cc:399-443, results written in place."""

    def __init__(self, layout: Layout, m: int, device="cuda"):
        lib = _lib.load()
        self.layout, self.m, self.device = layout, m, torch.device(device)
        self._p = ctypes.c_void_p()
        _lib.check(lib.omr_msg_plan_create(layout.n, layout.block_size, layout.num_lanes, layout.num_threads, m,
                                           ctypes.byref(self._p)), "omr_msg_plan_create")

    def run(self, bufs: Sequence[torch.Tensor], outs: Optional[Sequence[torch.Tensor]] = None, stream=None) -> int:
        L = self.layout
        outs = list(bufs) if outs is None else list(outs)
        if len(bufs) != self.m or len(outs) != self.m:
            raise ValueError(f"expected {self.m} worker buffers")
        for i, (b, o) in enumerate(zip(bufs, outs)):
            _check_f32(b, L.n, f"bufs[{i}]")
            _check_f32(o, L.n, f"outs[{i}]")
        maxr = ctypes.c_uint32()
        _lib.check(_lib.load().omr_msg_round_f32(self._p, _ptr_array(bufs), _ptr_array(outs), ctypes.byref(maxr),
                                                 _stream(stream)), "omr_msg_round_f32")
        return maxr.value

    def logs(self, worker: int) -> dict:
        """Copies of the wire logs: messages / replies [G, cap, 2*MESSAGE_SIZE] f32, imm / reply_imm [G, cap]
        (uint32 bits in int32), rounds [G]."""
        msg, imm, rep, rimm, rnd = (ctypes.c_void_p() for _ in range(5))
        cap = ctypes.c_uint32()
        _lib.check(_lib.load().omr_msg_logs(self._p, worker, ctypes.byref(msg), ctypes.byref(imm), ctypes.byref(rep),
                                            ctypes.byref(rimm), ctypes.byref(rnd), ctypes.byref(cap)), "omr_msg_logs")
        G, c, W = self.layout.num_threads * NUM_SLOTS, cap.value, 2 * MESSAGE_SIZE
        torch.cuda.synchronize(self.device)
        view = (lambda p, shape, t: torch.as_tensor(_DeviceView(p.value, shape, t), device=self.device).clone())
        return {"messages": view(msg, (G, c, W), "<f4"), "imm": view(imm, (G, c), "<i4"),
                "replies": view(rep, (G, c, W), "<f4"), "reply_imm": view(rimm, (G, c), "<i4"),
                "rounds": view(rnd, (G,), "<i4"), "cap": c}

    def close(self):
        if self._p:
            _lib.load().omr_msg_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown)
            pass
