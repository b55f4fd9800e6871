"""TEST SCAFFOLDING, not the product: a Python twin of the multi-rank round of csrc/omr_dist.hip (libomr_dist.so,
the product's driver), kept so the protocol runs on a GPU-less host over gloo (tests/test_dist.py, world 2-5, with
the oracle-backed tests/cpu_backend.py).  Same roles, shard bounds, packed-stream layout and pairing as the C++
round; a different implementation of the bookkeeping (block lists instead of prefix-addressed moves).

Roles (reference README.md:13-22, common.cc:381-383): with num_workers == world every rank r is worker r (its own
gradient tensor) and aggregator for shard r; with num_workers < world the ranks >= num_workers are dedicated
aggregators (the reference's separate servers) holding no tensor, aggregator j owning shard j.  A shard is a
contiguous range of rows (the reference shards message slots over aggregators by gs % n; a contiguous row range is
the same partition of the block space up to relabelling, and keeps every shard's packed streams in block order).

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

from omr import _lib, ops
from omr.layout import Layout


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

    def __init__(self, L: Layout, device=None, backend=None, comm=None, num_workers: Optional[int] = None):
        self.L = L
        self.comm = comm or TorchComm()
        self.rank, self.world = self.comm.rank, self.comm.world
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.M = self.world if num_workers is None else num_workers
        self.colocated = self.M == self.world
        self.A = self.world if self.colocated else self.world - self.M
        self.shard = self.rank if self.colocated else (self.rank - self.M if self.rank >= self.M else -1)
        self.be = backend or HipBackend(L, self.M, self.device)
        W, M, A, dev = self.world, self.M, self.A, self.device
        self.bounds = [s * L.rows // A for s in range(A + 1)]  # aggregator s owns rows [bounds[s], bounds[s+1])
        max_shard_rows = max(self.bounds[s + 1] - self.bounds[s] for s in range(A))
        shard_nb = max_shard_rows * L.num_lanes
        B = L.block_size
        i32, i64, f32 = torch.int32, torch.int64, torch.float32
        self.gathered = torch.zeros((W, L.rows), dtype=i64, device=dev)    # every rank's masks (aggregators: 0)
        self.masks_all = torch.zeros((M + 1, L.rows), dtype=i64, device=dev)  # workers ..., write set at [M]
        self.zero_mask = torch.zeros(L.rows, dtype=i64, device=dev)
        self.umask = torch.zeros((1, L.rows), dtype=i64, device=dev)
        self.prefix = torch.zeros((M + 1, L.rows + 1), dtype=i32, device=dev)
        self.my_list = torch.zeros(L.nb, dtype=i32, device=dev)
        self.full_list = torch.zeros(L.nb, dtype=i32, device=dev)
        self.shard_list = torch.zeros(shard_nb, dtype=i32, device=dev)
        self.count = torch.zeros(3, dtype=i32, device=dev)
        self.packed = torch.empty(L.n, dtype=f32, device=dev)          # own non-zero blocks, block order
        self.recv = torch.empty(M * shard_nb * B, dtype=f32, device=dev)  # shard contributions, worker-major
        self.recv_off = torch.zeros(M, dtype=i64, device=dev)
        self.sums = torch.empty(shard_nb * B, dtype=f32, device=dev)
        self.results = torch.empty(L.n, dtype=f32, device=dev)        # all shards' sums, shard-major
        self.bounds_t = torch.tensor(self.bounds, dtype=torch.long, device=dev)

    def agg_rank(self, s: int) -> int:
        return s if self.colocated else self.M + s

    def run(self, x: Optional[torch.Tensor], out: Optional[torch.Tensor] = None, ev=None,
            mode: int = 0) -> RoundResult:
        """One round.  A worker's result is scattered into `out` (default: x itself, the reference's in-place
        result, client.cc:89); an out-of-place `out` must already hold x's values outside the write set.  `ev` =
        optional (start, end) events around the worker-scan kernel.  mode 0 = all-reduce, 1 = reduce-scatter (stop
        at the aggregators: a co-located rank writes its shard of the write set into `out`, a dedicated aggregator
        keeps its packed sums in self.sums).  A dedicated aggregator passes x = None."""
        L, W, M, A, me, be, B = self.L, self.world, self.M, self.A, self.rank, self.be, self.L.block_size
        worker, sh = me < M, self.shard
        if worker and (x is None or x.numel() != L.n or x.dtype != torch.float32):
            raise ValueError("x must be float32[n]")
        out = x if out is None else out
        # 1. worker scan
        flags = nxt = None
        if worker:
            if ev is not None:
                ev[0].record()
            masks_r, flags, nxt = be.scan(x)
            if ev is not None:
                ev[1].record()
        else:
            masks_r = self.zero_mask
        # 2. every rank's row masks (a dedicated aggregator offers zeros)
        self.comm.all_gather_rows(self.gathered, masks_r)
        self.masks_all[:M].copy_(self.gathered[:M])
        # 3. write set (union + lane heads), union, aggregator chain, prefixes
        be.union(self.masks_all[:M], True, self.masks_all[M])
        be.union(self.masks_all[:M], False, self.umask[0])
        unext = be.next_offsets(self.umask[0])
        be.row_prefix(self.masks_all, self.prefix)
        cnt = self.prefix.index_select(1, self.bounds_t).cpu().tolist()  # [M+1][A+1], the one host sync
        per = [[cnt[a][s + 1] - cnt[a][s] for s in range(A)] for a in range(M + 1)]
        # 4. workers pack their non-zero blocks (block order = shard order) and send shard s's part to its aggregator
        sends = [None] * W
        recvs = [None] * W
        total_send = 0
        if worker:
            total_send = cnt[me][A]
            be.compact(masks_r, 0, L.rows, self.my_list, self.count[0:1])
            be.gather(x, self.my_list, total_send, self.packed)
            for s in range(A):
                off = cnt[me][s] - cnt[me][0]
                sends[self.agg_rank(s)] = self.packed[off * B:(off + per[me][s]) * B]
        roff = [0] * M
        if sh >= 0:
            acc = 0
            for w in range(M):
                roff[w] = acc
                recvs[w] = self.recv[acc * B:(acc + per[w][sh]) * B]
                acc += per[w][sh]
            if worker:  # a co-located rank's own contribution stays local
                recvs[me].copy_(sends[me])
            self.recv_off.copy_(torch.tensor(roff, dtype=torch.int64), non_blocking=False)
        self.comm.exchange([t if p != me else None for p, t in enumerate(sends)],
                           [t if p != me else None for p, t in enumerate(recvs)])
        # 5. aggregator: rank-order sums of this shard's write set
        nres = per[M]
        if sh >= 0:
            r0, r1 = self.bounds[sh], self.bounds[sh + 1]
            be.compact(self.masks_all[M], r0, r1, self.shard_list, self.count[1:2])
            be.sparse_sum(self.recv, self.recv_off, self.masks_all[:M], self.prefix, r0, self.shard_list, nres[sh],
                          self.sums)
        sent = total_send - (per[me][me] if worker and self.colocated else 0)
        if mode == 1:  # reduce-scatter: the aggregator keeps its shard
            if worker and sh >= 0:
                be.scatter(self.sums, self.shard_list, nres[sh], out)
            return RoundResult(flags, masks_r, nxt, unext, nres[sh] if sh >= 0 else 0, sent)
        # 6. results back to every worker, scattered in place
        res_off = [cnt[M][s] - cnt[M][0] for s in range(A)]
        sends = [None] * W
        recvs = [None] * W
        if sh >= 0:
            for w in range(M):
                sends[w] = self.sums[:nres[sh] * B]
        if worker:
            for s in range(A):
                recvs[self.agg_rank(s)] = self.results[res_off[s] * B:(res_off[s] + nres[s]) * B]
            if sh >= 0:
                recvs[me].copy_(self.sums[:nres[sh] * B])
        self.comm.exchange([t if p != me else None for p, t in enumerate(sends)],
                           [t if p != me else None for p, t in enumerate(recvs)])
        total_res = cnt[M][A]
        if worker:
            be.compact(self.masks_all[M], 0, L.rows, self.full_list, self.count[2:3])
            be.scatter(self.results, self.full_list, total_res, out)
        return RoundResult(flags, masks_r, nxt, unext, total_res, sent)
