"""ctypes binding of the C++ multi-rank round (include/omr_dist.h, libomr_dist.so).

`CppSparseAllreduce` is one rank of the product's OmniReduce round: the whole round — kernels,
block-count sync, RCCL all-gather and grouped send/recv — is driven from C++ (omr_dist.hip).  Python only
bootstraps the RCCL communicator: rank 0's unique id is broadcast over the torch.distributed group the job was
launched with (torch.distributed.run), standing in for the reference's TCP bootstrap.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
import torch.distributed as dist

from . import _lib
from .layout import Layout

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libomr_dist.so")
UNIQUE_ID_BYTES = 128
_dl = None


def load():
    global _dl
    if _dl is not None:
        return _dl
    _lib.load()  # libomr.so first (libomr_dist.so links it), after torch's HIP/RCCL runtimes
    if not os.path.exists(LIB_PATH):
        raise _lib.OmrError(f"libomr_dist.so not found at {LIB_PATH}: build with `make -C omnireduce-rdma-demo_amd`")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "omr_dist_last_error": (ctypes.c_char_p, []),
        "omr_dist_unique_id": (i, [vp]),
        "omr_dist_create_rccl": (i, [vp, i, i, vp]),
        "omr_dist_ipc_unique_id": (i, [vp]),
        "omr_dist_create_ipc": (i, [vp, i, i, vp]),
        "omr_local_board_create": (vp, [i]),
        "omr_local_board_destroy": (None, [vp]),
        "omr_dist_create_local": (i, [vp, i, vp]),
        "omr_dist_rank": (i, [vp]),
        "omr_dist_world": (i, [vp]),
        "omr_dist_destroy": (i, [vp]),
        "omr_dist_allgather": (i, [vp, vp, vp, ctypes.c_size_t, vp]),
        "omr_dist_exchange": (i, [vp, vp, vp, vp, vp, vp]),
        "omr_dist_inject_fault": (i, [vp, ctypes.c_int64]),
        "omr_dist_inject_allgather_fault": (i, [vp]),
        "omr_dist_abort": (i, [vp]),
        "omr_dist_aborted": (i, [vp]),
        "omr_dist_set_timeout": (i, [vp, ctypes.c_int64]),
        "omr_dist_poll": (i, [vp]),
        "omr_ar_plan_wait": (i, [vp, vp]),
        "omr_ar_plan_failed": (i, [vp]),
        "omr_ar_plan_host_stats": (i, [vp, vp, vp, i]),
        "omr_ar_plan_create": (i, [vp, u64, u32, u32, u32, vp]),
        "omr_ar_plan_destroy": (i, [vp]),
        "omr_ar_plan_create_roles": (i, [vp, u32, u64, u32, u32, u32, vp]),
        "omr_ar_plan_shard": (i, [vp, vp, vp, vp, vp, vp]),
        "omr_sparse_allreduce_f32": (i, [vp, vp, vp, vp, vp, vp, vp, vp, vp]),
        "omr_sparse_round_f32": (i, [vp, vp, vp, vp, vp, vp, i, vp, vp, vp]),
        "omr_ar_plan_join": (i, [vp, vp]),
        "omr_ar_plan_set_side_streams": (i, [vp, i]),
        "omr_ar_plan_side_streams": (i, [vp]),
        "omr_ar_plan_set_queue_check": (i, [vp, i]),
        "omr_ar_plan_queue_report": (i, [vp, vp, vp, vp]),
        "omr_ar_plan_fused_pack": (i, [vp]),
        "omr_ar_plan_device_bytes": (u64, [vp]),
        "omr_dist_test_world1_round": (i, [vp, i]),
        "omr_sparse_buckets_f32": (i, [vp, vp, u64, i, vp, vp, vp]),
        "omr_msgd_plan_create": (i, [vp, u32, u64, u32, u32, u32, vp]),
        "omr_msgd_plan_destroy": (i, [vp]),
        "omr_msgd_round_f32": (i, [vp, vp, vp, vp, vp]),
        "omr_msgd_logs": (i, [vp, u32, vp, vp, vp, vp, vp, vp]),
        "omr_ar_plan_exchange_time": (i, [vp, vp, vp, vp]),
        "omr_ar_plan_timings": (i, [vp, vp, vp, vp, vp, vp]),
        "omr_ar_plan_stage_timings": (i, [vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    _dl = L
    return L


def _check(rc: int, what: str):
    if rc != 0:
        raise _lib.OmrError(f"{what} failed (rc={rc}): {load().omr_dist_last_error().decode(errors='replace')}")


def ipc_unique_id() -> bytes:
    """A fresh id for omr_dist_create_ipc (names the shared board); hand it to every rank out of band."""
    uid = (ctypes.c_ubyte * UNIQUE_ID_BYTES)()
    _check(load().omr_dist_ipc_unique_id(uid), "omr_dist_ipc_unique_id")
    return bytes(uid)


class CppSparseAllreduce:
    """One rank of the C++ round.  transport "rccl" (default): one process per GPU, the torch.distributed default
    group supplies rank/world and the unique-id broadcast.  transport "ipc": ranks are processes of one node sharing
    any GPUs (omr_dist_create_ipc); rank, world and the id (ipc_unique_id() of one rank) are passed in.  transport
    "local1": a group of one rank (the round with no peers), e.g. for the single-GPU host-resident bench.  transport
    "rccl1": a one-rank RCCL communicator made in this process (no torch.distributed group): the N>1 bench path's
    round with no peers, e.g. bench.py's world-1 round line."""

    def __init__(self, L: Layout, device, group=None, transport: str = "rccl", uid: Optional[bytes] = None,
                 rank: Optional[int] = None, world: Optional[int] = None, num_workers: Optional[int] = None):
        """num_workers < world: ranks >= num_workers are dedicated aggregators (omr_ar_plan_create_roles): they
        call run() with x = None."""
        D = load()
        self.L = L
        self.device = torch.device(device)
        self._d = ctypes.c_void_p()
        self._board = None
        if transport == "local1":  # a one-rank group (loopback transport): the round without peers
            rank, world = 0, 1
            self._board = D.omr_local_board_create(1)
            _check(D.omr_dist_create_local(self._board, 0, ctypes.byref(self._d)), "omr_dist_create_local")
        elif transport == "rccl1":
            rank, world = 0, 1
            uid = (ctypes.c_ubyte * UNIQUE_ID_BYTES)()
            _check(D.omr_dist_unique_id(uid), "omr_dist_unique_id")
            _check(D.omr_dist_create_rccl(uid, 0, 1, ctypes.byref(self._d)), "omr_dist_create_rccl")
        elif transport == "ipc":
            if uid is None or rank is None or world is None:
                raise ValueError("the ipc transport needs uid, rank and world")
            buf = (ctypes.c_ubyte * UNIQUE_ID_BYTES).from_buffer_copy(uid.ljust(UNIQUE_ID_BYTES, b"\0"))
            _check(D.omr_dist_create_ipc(buf, rank, world, ctypes.byref(self._d)), "omr_dist_create_ipc")
        else:
            rank, world = dist.get_rank(group), dist.get_world_size(group)
            uidt = torch.zeros(UNIQUE_ID_BYTES, dtype=torch.uint8)
            if rank == 0:
                _check(D.omr_dist_unique_id(uidt.data_ptr()), "omr_dist_unique_id")
            bdev = self.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            t = uidt.to(bdev)
            dist.broadcast(t, 0, group=group)
            uidt.copy_(t.cpu())
            _check(D.omr_dist_create_rccl(uidt.data_ptr(), rank, world, ctypes.byref(self._d)), "omr_dist_create_rccl")
        self._p = ctypes.c_void_p()
        nw = world if num_workers is None else num_workers
        self.rank, self.world, self.num_workers = rank, world, nw
        self._plan()

    def _plan(self):
        L = self.L
        _check(load().omr_ar_plan_create_roles(self._d, self.num_workers, L.n, L.block_size, L.num_lanes,
                                               L.num_threads, ctypes.byref(self._p)), "omr_ar_plan_create_roles")

    @property
    def fused_pack(self) -> bool:
        """The worker scan packs the exchange's blocks itself (omr_ar_plan_fused_pack)."""
        return bool(load().omr_ar_plan_fused_pack(self._p))

    @property
    def device_bytes(self) -> int:
        """Device memory the plan holds (omr_ar_plan_device_bytes)."""
        return int(load().omr_ar_plan_device_bytes(self._p))

    def test_world1_round(self, on: bool = True):
        """Test hook (omr_dist_test_world1_round): a one-rank group runs the multi-rank round's code path (all-gather,
        plan, exchange) and an RCCL transport issues its collectives as RCCL calls.  Plans made after it also take the
        N > 1 stream layout (a plan stream and an exchange stream; replan() to apply it to this engine's plan)."""
        _check(load().omr_dist_test_world1_round(self._d, int(on)), "omr_dist_test_world1_round")

    def set_side_streams(self, n: int):
        """1 or 2 side streams for the asynchronous rounds (omr_ar_plan_set_side_streams); returns the previous count."""
        old = int(load().omr_ar_plan_side_streams(self._p))
        _check(load().omr_ar_plan_set_side_streams(self._p, int(n)), "omr_ar_plan_set_side_streams")
        return old

    @property
    def side_streams(self) -> int:
        return int(load().omr_ar_plan_side_streams(self._p))

    def set_queue_check(self, on: bool = True):
        """Check (default) or not the side streams' hardware queues against the caller's stream before its first
        asynchronous round (omr_ar_plan_set_queue_check)."""
        _check(load().omr_ar_plan_set_queue_check(self._p, int(on)), "omr_ar_plan_set_queue_check")

    def queue_report(self) -> dict:
        """{"disjoint": 1 / 0 / -1 (not checked yet), "probes": n, "replaced": n} (omr_ar_plan_queue_report)."""
        d, pr, rp = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(load().omr_ar_plan_queue_report(self._p, ctypes.byref(d), ctypes.byref(pr), ctypes.byref(rp)),
               "omr_ar_plan_queue_report")
        return {"disjoint": d.value, "probes": pr.value, "replaced": rp.value}

    def replan(self, L: Optional[Layout] = None):
        """Destroy the plan and make a new one on the same transport, of the same shape or of layout L (collective: every
        rank calls it).  The new plan's buffers may land at the old ones' addresses, or reuse the transport's parked
        exported ones (IPC): the transport must not reuse what it cached about the freed ones (their handles)."""
        load().omr_ar_plan_destroy(self._p)
        self._p = ctypes.c_void_p()
        if L is not None:
            self.L = L
        self._plan()

    ALLREDUCE, REDUCE_SCATTER, DENSE_REDUCE_SCATTER, ASYNC, TIME_EXCHANGE, DEFER = 0, 1, 2, 0x100, 0x200, 0x400
    THREAD = 0x800

    def run(self, x: Optional[torch.Tensor], out: Optional[torch.Tensor] = None, ev=None, flags=None, next_offsets=None,
            union_next=None, mode: int = 0, async_: bool = False, time_exchange: bool = False,
            defer: bool = False, thread: bool = False, counts: bool = True):
        """mode 0: all-reduce (every worker gets every shard's sums); 1: reduce-scatter (stop at the
        aggregators: `out` gets this rank's shard sums only); 2: the dense stand-in (the whole tensor reduce-scattered
        by RCCL, every block).  async_: only the worker scan runs on the caller's stream; the bookkeeping, the
        exchange and the sums run on the plan's side stream, overlapping the next calls' scans; `out` (and
        union_next) are ready after join().  (A one-rank group's round is its worker scan alone, on the caller's
        stream.)  time_exchange: bracket the worker scan and the worker ->
        aggregator exchange with timing events (read with timings() / exchange_time()).  defer: OMR_ROUND_DEFER,
        this round's exchange is issued two calls later (or by a call without the flag, or join()); the returned
        counts are those of the round whose exchange this call issued.  thread: OMR_ROUND_THREAD (implies async_),
        the plan's progress thread issues everything after the worker scan; the returned counts are 0.
        counts=False: ask for no counts (returns (None, None)); a one-rank round then does not wait at all."""
        if thread:
            mode |= self.THREAD
        if defer:
            mode |= self.DEFER
        if async_:
            mode |= self.ASYNC
        if time_exchange:
            mode |= self.TIME_EXCHANGE
        out = x if out is None else out
        sent, uni = ctypes.c_uint64(), ctypes.c_uint64()
        st = torch.cuda.current_stream(self.device)
        if ev is not None:  # the round starts with the worker scan kernel on this stream
            ev[0].record(st)
        ptr = (lambda t: t.data_ptr() if t is not None else None)
        _check(load().omr_sparse_round_f32(self._p, ptr(x), ptr(out), ptr(flags), ptr(next_offsets),
                                           ptr(union_next), mode, ctypes.byref(sent) if counts else None,
                                           ctypes.byref(uni) if counts else None, st.cuda_stream),
               "omr_sparse_round_f32")
        if ev is not None:
            ev[1].record(st)
        return (sent.value, uni.value) if counts else (None, None)

    def shard(self):
        """(shard, row_begin, row_end, sums, num_blocks) of this rank (omr_ar_plan_shard); `sums` is a device pointer
        (a dedicated aggregator's last shard sums, write-set order) or None."""
        sh, r0, r1 = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        sums, nb = ctypes.c_void_p(), ctypes.c_uint64()
        _check(load().omr_ar_plan_shard(self._p, ctypes.byref(sh), ctypes.byref(r0), ctypes.byref(r1),
                                        ctypes.byref(sums), ctypes.byref(nb)), "omr_ar_plan_shard")
        return sh.value, r0.value, r1.value, sums.value, nb.value

    def run_buckets(self, buf: torch.Tensor, mode: int = 0, stream=None):
        """The whole tensor `buf` (numel a multiple of the layout's n) reduced in place, one pipelined round per
        bucket of L.n floats (omr_sparse_buckets_f32).  buf on the device, or in pinned host memory (staged: returns
        when the host buffer holds the result).  Returns (sent blocks, union blocks) summed over the buckets."""
        if buf.dtype != torch.float32 or not buf.is_contiguous() or buf.numel() % self.L.n:
            raise ValueError("buf must be a contiguous float32 tensor of a multiple of the bucket's n")
        if not buf.is_cuda and not buf.is_pinned():
            raise ValueError("a host buffer must be pinned (pin_memory())")
        sent, uni = ctypes.c_uint64(), ctypes.c_uint64()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(load().omr_sparse_buckets_f32(self._p, buf.data_ptr(), buf.numel(), mode, ctypes.byref(sent),
                                             ctypes.byref(uni), st.cuda_stream), "omr_sparse_buckets_f32")
        return sent.value, uni.value

    def exchange_time(self):
        """(ms, bytes sent, bytes received) of the last round run with time_exchange=True (waits for it)."""
        ms, bo, bi = ctypes.c_float(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(load().omr_ar_plan_exchange_time(self._p, ctypes.byref(ms), ctypes.byref(bo), ctypes.byref(bi)),
               "omr_ar_plan_exchange_time")
        return ms.value, bo.value, bi.value

    def timings(self):
        """Means over the rounds run with time_exchange=True since the last call (omr_ar_plan_timings): (worker scan
        ms, exchange ms, bytes out per rank, bytes in per rank, timed rounds)."""
        sm, xm, bo, bi, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        _check(load().omr_ar_plan_timings(self._p, ctypes.byref(sm), ctypes.byref(xm), ctypes.byref(bo),
                                          ctypes.byref(bi), ctypes.byref(n)), "omr_ar_plan_timings")
        return sm.value, xm.value, bo.value, bi.value, n.value

    STAGES = ("scan", "bookkeeping", "exchange", "aggregate")

    def stage_timings(self):
        """As timings(), per stage (omr_ar_plan_stage_timings): ({stage: mean ms} over STAGES, bytes out per rank,
        bytes in per rank, timed rounds)."""
        ms = (ctypes.c_float * len(self.STAGES))()
        bo, bi, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        _check(load().omr_ar_plan_stage_timings(self._p, ms, ctypes.byref(bo), ctypes.byref(bi), ctypes.byref(n)),
               "omr_ar_plan_stage_timings")
        return dict(zip(self.STAGES, list(ms))), bo.value, bi.value, n.value

    def join(self, stream=None):
        """Make `stream` (default: the current stream) wait for every asynchronous round issued so far."""
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(load().omr_ar_plan_join(self._p, st.cuda_stream), "omr_ar_plan_join")

    def wait(self, stream=None):
        """Join every round issued so far into `stream` and wait on the host until it has run them, within the
        transport's deadline (omr_ar_plan_wait): raises instead of blocking on a peer that is stuck or gone (the
        transport is then aborted)."""
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(load().omr_ar_plan_wait(self._p, st.cuda_stream), "omr_ar_plan_wait")

    def set_timeout(self, ms: int):
        """The deadline of every host-side wait of the transport and its rounds (omr_dist_set_timeout)."""
        _check(load().omr_dist_set_timeout(self._d, int(ms)), "omr_dist_set_timeout")

    def abort(self):
        """Abort the transport (omr_dist_abort): RCCL's communicators are aborted, loopback / IPC peers' waits on this
        rank end at once; every later call fails.  For a rank that cannot finish its part of a round."""
        if self._d:
            _check(load().omr_dist_abort(self._d), "omr_dist_abort")

    @property
    def aborted(self) -> bool:
        return bool(self._d) and bool(load().omr_dist_aborted(self._d))

    def host_stats(self, reset: bool = True):
        """(microseconds the calling thread spent blocked inside the plan's calls, number of waits) since the last
        reset (omr_ar_plan_host_stats): a round's host issue time is its call time minus the blocked time."""
        us, n = ctypes.c_double(), ctypes.c_uint64()
        _check(load().omr_ar_plan_host_stats(self._p, ctypes.byref(us), ctypes.byref(n), int(reset)),
               "omr_ar_plan_host_stats")
        return us.value, n.value

    @property
    def failed(self) -> int:
        """The plan's first failure code (0: none)."""
        return int(load().omr_ar_plan_failed(self._p)) if self._p else 0

    def inject_allgather_fault(self):
        """Test hook (omr_dist_inject_allgather_fault): the next all-gather fails (a round failing in its first half)."""
        _check(load().omr_dist_inject_allgather_fault(self._d), "omr_dist_inject_allgather_fault")

    def inject_fault(self, after_pieces: int = 0):
        """Test hook (omr_dist_inject_fault): the next exchange fails after issuing `after_pieces` pieces."""
        _check(load().omr_dist_inject_fault(self._d, after_pieces), "omr_dist_inject_fault")

    def allgather(self, src: torch.Tensor, dst: torch.Tensor, stream=None):
        """The transport's all-gather of src.nbytes per rank into dst (omr_dist_allgather)."""
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        _check(load().omr_dist_allgather(self._d, src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size(),
                                         st.cuda_stream), "omr_dist_allgather")

    def exchange(self, sends, recvs, stream=None) -> int:
        """One grouped exchange (omr_dist_exchange): sends[p] to peer p, recvs[p] from peer p (tensors or None).
        Returns the C return code instead of raising (the fault-injection tests look at it)."""
        W = self.world
        sp, sb = (ctypes.c_void_p * W)(), (ctypes.c_size_t * W)()
        rp, rb = (ctypes.c_void_p * W)(), (ctypes.c_size_t * W)()
        for p in range(W):
            if sends[p] is not None:
                sp[p], sb[p] = sends[p].data_ptr(), sends[p].numel() * sends[p].element_size()
            if recvs[p] is not None:
                rp[p], rb[p] = recvs[p].data_ptr(), recvs[p].numel() * recvs[p].element_size()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        return load().omr_dist_exchange(self._d, sp, sb, rp, rb, st.cuda_stream)

    def close(self):
        """Destroy the plan and the transport; returns their codes (0, 0) when both released everything (after an
        abort, OMR_ETIMEDOUT where the device was still busy past the deadline and device memory was left allocated)."""
        D = load()
        rcs = [0, 0]
        if self._p:
            rcs[0] = D.omr_ar_plan_destroy(self._p)
            self._p = ctypes.c_void_p()
        if self._d:
            rcs[1] = D.omr_dist_destroy(self._d)
            self._d = ctypes.c_void_p()
        if self._board:
            D.omr_local_board_destroy(self._board)
            self._board = None
        return tuple(rcs)
