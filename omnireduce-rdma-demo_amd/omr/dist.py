"""N-GPU sparse all-reduce: OmniReduce's worker -> aggregator -> worker round with the RDMA hop replaced by
RCCL over xGMI (one process per GPU, torch.distributed backend "nccl" = RCCL).

Roles (reference README.md:13-22, common.cc:381-383): every rank r is worker r (its own gradient tensor) and
aggregator for shard r, a contiguous range of rows (the reference shards message slots over aggregators by
gs % n; a contiguous row range is the same partition of the block space up to relabelling, and keeps every
shard's packed streams in increasing block order).

One round (= one bench step at N > 1):
  1. worker scan of the local tensor (HIP: flags, row masks, the worker's next-offset chain);
  2. all-gather of the row masks (8 B per 64 KiB row) -> every rank knows every worker's non-zero set;
  3. union masks (the aggregator's min_next chain runs over them, server.cc:86-96) and the write set
     (union + lane heads, client.cc:201-205), exclusive row prefixes of every mask (HIP);
  4. each worker packs its non-zero blocks (common.cc:405-407) and sends shard s's part to aggregator s,
     grouped RCCL send/recv;
  5. aggregator s sums its shard in rank order from a zeroed accumulator (server.cc:97-98, :148-150), locating
     every contribution through the prefixes (HIP, k_sparse_sum);
  6. the shard sums go back to every worker (grouped send/recv, server.cc:162) and are scattered in place
     (client.cc:89).
The only host synchronisation is one small device->host copy of per-shard block counts (RCCL needs buffer
sizes on the host); no index list crosses a link.

Compute goes through a backend object; the product backend is HipBackend (libomr.so).  Tests inject a CPU
backend (tests/cpu_backend.py, built on the oracle) to run the same protocol over gloo on a GPU-less host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib
from .layout import Layout
from . import ops


# ------------------------------------------------------------------ compute backend (product: HIP)

class HipBackend:
    """libomr.so kernels on device tensors; allocates its workspaces once."""

    def __init__(self, L: Layout, world: int, device):
        self.L, self.device = L, device
        self.scan_plan = ops.ScanSumPlan(L, 1, with_flags=True, with_next=True, device=device)
        lib = _lib.load()
        self.prefix_ws = torch.empty(lib.omr_prefix_workspace_bytes(L.rows, world + 1), dtype=torch.uint8,
                                     device=device)
        self.compact_ws = torch.empty(lib.omr_compact_workspace_bytes(L.rows), dtype=torch.uint8, device=device)
        self.unext = torch.empty((1, L.nb), dtype=torch.int32, device=device)

    def scan(self, x):
        r = self.scan_plan.run([x], None)
        return r.masks[0], r.flags[0], r.next_offsets[0]

    def union(self, masks_all, heads: bool, out):
        L = self.L
        _lib.check(_lib.load().omr_mask_union(masks_all.data_ptr(), masks_all.shape[0], L.rows, L.rows_per_part,
                                              L.num_lanes, int(heads), out.data_ptr(), ops._stream()),
                   "omr_mask_union")
        return out

    def next_offsets(self, mask):
        L = self.L
        _lib.check(_lib.load().omr_next_offsets(mask.data_ptr(), 1, L.n, L.block_size, L.num_lanes, L.num_threads,
                                                self.unext.data_ptr(), ops._stream()), "omr_next_offsets")
        return self.unext[0]

    def row_prefix(self, masks, prefix):
        _lib.check(_lib.load().omr_row_prefix(masks.data_ptr(), masks.shape[0], self.L.rows, prefix.data_ptr(),
                                              self.prefix_ws.data_ptr(), self.prefix_ws.numel(), ops._stream()),
                   "omr_row_prefix")
        return prefix

    def compact(self, mask, r0, r1, out_list, out_count):
        _lib.check(_lib.load().omr_compact(mask.data_ptr(), r0, r1, self.L.num_lanes, out_list.data_ptr(),
                                           out_count.data_ptr(), self.compact_ws.data_ptr(), self.compact_ws.numel(),
                                           ops._stream()), "omr_compact")

    def gather(self, x, lst, k, packed):
        ops.gather_blocks(x, lst, k, self.L.block_size, packed)

    def sparse_sum(self, recv, recv_off, masks_all, prefix, row_begin, lst, k, out):
        if k == 0:
            return
        L = self.L
        _lib.check(_lib.load().omr_sparse_block_sum_f32(recv.data_ptr(), recv_off.data_ptr(), masks_all.data_ptr(),
                                                        masks_all.shape[0], L.rows, prefix.data_ptr(), row_begin,
                                                        L.num_lanes, lst.data_ptr(), k, L.block_size, out.data_ptr(),
                                                        ops._stream()), "omr_sparse_block_sum_f32")

    def scatter(self, packed, lst, k, dst):
        ops.scatter_blocks(packed, lst, k, self.L.block_size, dst)


# ------------------------------------------------------------------ communication

class TorchComm:
    """torch.distributed collectives on the backend's tensors (RCCL on GPU tensors, gloo on CPU tensors)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.nccl = dist.get_backend(group) == "nccl"

    def all_gather_rows(self, out, inp):
        if self.nccl:
            dist.all_gather_into_tensor(out.view(-1), inp, group=self.group)
        else:
            parts = list(out.unbind(0))
            dist.all_gather(parts, inp, group=self.group)

    def exchange(self, sends: List[Optional[torch.Tensor]], recvs: List[Optional[torch.Tensor]]):
        """Grouped point-to-point: sends[p] to peer p, recvs[p] from peer p (None or empty = nothing)."""
        p2p = []
        for p in range(self.world):
            if p == self.rank:
                continue
            if recvs[p] is not None and recvs[p].numel() > 0:
                p2p.append(dist.P2POp(dist.irecv, recvs[p], p, self.group))
            if sends[p] is not None and sends[p].numel() > 0:
                p2p.append(dist.P2POp(dist.isend, sends[p], p, self.group))
        if p2p:
            for req in dist.batch_isend_irecv(p2p):
                req.wait()


# ------------------------------------------------------------------ the round

@dataclass
class RoundResult:
    flags: torch.Tensor  # worker flags [nb]
    masks: torch.Tensor  # worker row masks [rows]
    next_offsets: torch.Tensor  # worker chain [nb] (uint32 bits)
    union_next: torch.Tensor  # aggregator chain [nb] (uint32 bits)
    union_blocks: int  # blocks in the write set (union + lane heads)
    sent_blocks: int  # blocks this worker sent to other aggregators


class SparseAllreduce:
    """In-place sparse all-reduce of one fp32 gradient per rank (OmniReduce round, see module docstring)."""

    def __init__(self, L: Layout, device=None, backend=None, comm=None):
        self.L = L
        self.comm = comm or TorchComm()
        self.rank, self.world = self.comm.rank, self.comm.world
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.be = backend or HipBackend(L, self.world, self.device)
        N, dev = self.world, self.device
        self.bounds = [s * L.rows // N for s in range(N + 1)]  # aggregator s owns rows [bounds[s], bounds[s+1])
        max_shard_rows = max(self.bounds[s + 1] - self.bounds[s] for s in range(N))
        shard_nb = max_shard_rows * L.num_lanes
        B = L.block_size
        i32, i64, f32 = torch.int32, torch.int64, torch.float32
        self.masks_all = torch.zeros((N + 1, L.rows), dtype=i64, device=dev)  # workers ..., write set at [N]
        self.umask = torch.zeros((1, L.rows), dtype=i64, device=dev)
        self.prefix = torch.zeros((N + 1, L.rows + 1), dtype=i32, device=dev)
        self.my_list = torch.zeros(L.nb, dtype=i32, device=dev)
        self.full_list = torch.zeros(L.nb, dtype=i32, device=dev)
        self.shard_list = torch.zeros(shard_nb, dtype=i32, device=dev)
        self.count = torch.zeros(3, dtype=i32, device=dev)
        self.packed = torch.empty(L.n, dtype=f32, device=dev)          # own non-zero blocks, block order
        self.recv = torch.empty(N * shard_nb * B, dtype=f32, device=dev)  # shard contributions, worker-major
        self.recv_off = torch.zeros(N, dtype=i64, device=dev)
        self.sums = torch.empty(shard_nb * B, dtype=f32, device=dev)
        self.results = torch.empty(L.n, dtype=f32, device=dev)        # all shards' sums, shard-major
        self.bounds_t = torch.tensor(self.bounds, dtype=torch.long, device=dev)

    def run(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, ev=None, mode: int = 0) -> RoundResult:
        """One round.  The result is scattered into `out` (default: x itself, the reference's in-place result,
        client.cc:89); an out-of-place `out` must already hold x's values outside the write set.  `ev` =
        optional (start, end) events recorded around the worker-scan kernel.  mode 0 = all-reduce, 1 =
        reduce-scatter (stop at the aggregators: only this rank's shard of the write set is written)."""
        L, N, me, be, B = self.L, self.world, self.rank, self.be, self.L.block_size
        if x.numel() != L.n or x.dtype != torch.float32:
            raise ValueError("x must be float32[n]")
        out = x if out is None else out
        # 1. worker scan
        if ev is not None:
            ev[0].record()
        masks_r, flags, nxt = be.scan(x)
        if ev is not None:
            ev[1].record()
        # 2. every worker's row masks
        self.comm.all_gather_rows(self.masks_all[:N], masks_r)
        # 3. write set (union + lane heads), union, aggregator chain, prefixes
        be.union(self.masks_all[:N], True, self.masks_all[N])
        be.union(self.masks_all[:N], False, self.umask[0])
        unext = be.next_offsets(self.umask[0])
        be.row_prefix(self.masks_all, self.prefix)
        cnt = self.prefix.index_select(1, self.bounds_t).cpu().tolist()  # [N+1][N+1], the one host sync
        per = [[cnt[a][s + 1] - cnt[a][s] for s in range(N)] for a in range(N + 1)]
        # 4. pack own non-zero blocks (block order = shard order) and exchange with the aggregators
        total_send = cnt[me][N]
        be.compact(masks_r, 0, L.rows, self.my_list, self.count[0:1])
        be.gather(x, self.my_list, total_send, self.packed)
        send_off = [cnt[me][s] - cnt[me][0] for s in range(N)]
        recv_blocks = [per[w][me] for w in range(N)]
        roff = [sum(recv_blocks[:w]) for w in range(N)]
        sends = [self.packed[send_off[s] * B:(send_off[s] + per[me][s]) * B] for s in range(N)]
        recvs = [self.recv[roff[w] * B:(roff[w] + recv_blocks[w]) * B] for w in range(N)]
        recvs[me].copy_(sends[me])
        self.recv_off.copy_(torch.tensor(roff, dtype=torch.int64), non_blocking=False)
        self.comm.exchange(sends, recvs)
        # 5. aggregator: rank-order sums of this shard's write set
        r0, r1 = self.bounds[me], self.bounds[me + 1]
        nres = per[N]
        be.compact(self.masks_all[N], r0, r1, self.shard_list, self.count[1:2])
        be.sparse_sum(self.recv, self.recv_off, self.masks_all[:N], self.prefix, r0, self.shard_list, nres[me],
                      self.sums)
        if mode == 1:  # reduce-scatter: the aggregator keeps its shard (sums scattered in place into `out`)
            be.scatter(self.sums, self.shard_list, nres[me], out)
            return RoundResult(flags, masks_r, nxt, unext, nres[me], total_send - per[me][me])
        # 6. results back to every worker, scattered in place
        res_off = [cnt[N][s] - cnt[N][0] for s in range(N)]
        my_sums = self.sums[:nres[me] * B]
        res_recvs = [self.results[res_off[s] * B:(res_off[s] + nres[s]) * B] for s in range(N)]
        res_recvs[me].copy_(my_sums)
        self.comm.exchange([my_sums if p != me else None for p in range(N)], res_recvs)
        total_res = cnt[N][N]
        be.compact(self.masks_all[N], 0, L.rows, self.full_list, self.count[2:3])
        be.scatter(self.results, self.full_list, total_res, out)
        return RoundResult(flags, masks_r, nxt, unext, total_res, total_send - per[me][me])
