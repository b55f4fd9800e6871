"""Test-only stand-ins for the dist twin (tests/dist_twin.py): a CPU compute backend built on the oracle, and a host-staged comm that lets
several processes share one GPU over gloo.  Neither is reachable from the product path (dist_twin uses
HipBackend + TorchComm unless a caller injects these)."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

import oracle


def _np(t):
    return t.detach().cpu().numpy()


class CpuBackend:
    """Same interface as dist_twin.HipBackend, computed on the host with the oracle (tensors stay on CPU)."""

    def __init__(self, L, world, device="cpu"):
        self.L = L

    def _flags_from_mask(self, mask):
        m = _np(mask).view(np.uint64)
        bits = ((m[:, None] >> np.arange(self.L.num_lanes, dtype=np.uint64)[None, :]) & np.uint64(1))
        return np.ascontiguousarray(bits.reshape(-1).astype(np.int32))

    def scan(self, x):
        L = self.L
        f = oracle.flags_from_data(np.ascontiguousarray(_np(x)), L.block_size)
        masks = oracle.row_masks(f, L.num_lanes).view(np.int64)
        nxt = oracle.next_offsets(f, L.n, L.block_size, L.num_lanes, L.num_threads).view(np.int32)
        return torch.from_numpy(masks.copy()), torch.from_numpy(f), torch.from_numpy(nxt.copy())

    def union(self, masks_all, heads, out):
        L = self.L
        u = np.bitwise_or.reduce(_np(masks_all).view(np.uint64), axis=0)
        if heads:
            lane_bits = np.uint64((1 << L.num_lanes) - 1) if L.num_lanes < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
            u[:: L.rows_per_part] |= lane_bits
        out.copy_(torch.from_numpy(u.view(np.int64).copy()))
        return out

    def next_offsets(self, mask):
        L = self.L
        f = self._flags_from_mask(mask)
        return torch.from_numpy(oracle.next_offsets(f, L.n, L.block_size, L.num_lanes, L.num_threads).view(np.int32))

    def row_prefix(self, masks, prefix):
        m = _np(masks).view(np.uint64)
        pc = np.vectorize(lambda v: bin(int(v)).count("1"))(m) if m.size else m
        pre = np.zeros((m.shape[0], m.shape[1] + 1), dtype=np.int32)
        pre[:, 1:] = np.cumsum(pc, axis=1)
        prefix.copy_(torch.from_numpy(pre))
        return prefix

    def compact(self, mask, r0, r1, out_list, out_count):
        f = self._flags_from_mask(mask)
        NB = self.L.num_lanes
        idx = np.nonzero(f[r0 * NB:r1 * NB])[0] + r0 * NB
        out_list[: idx.size] = torch.from_numpy(idx.astype(np.int32))
        out_count.fill_(idx.size)

    def gather(self, x, lst, k, packed):
        B = self.L.block_size
        if k:
            idx = _np(lst[:k]).astype(np.int64)
            packed[: k * B] = torch.from_numpy(_np(x).reshape(-1, B)[idx].reshape(-1))

    def sparse_sum(self, recv, recv_off, masks_all, prefix, row_begin, lst, k, out):
        """Rank-order sum from a zeroed accumulator (server.cc:97-98, :148-150); contributions located by
        counting each worker's set bits before the block inside the shard."""
        L, B = self.L, self.L.block_size
        rv = _np(recv).reshape(-1, B)
        offs = _np(recv_off)
        m = _np(masks_all).view(np.uint64)
        ids = _np(lst[:k]).astype(np.int64)
        res = np.zeros((k, B), dtype=np.float32)
        for w in range(m.shape[0]):
            f = self._flags_from_mask(masks_all[w])
            start = row_begin * L.num_lanes
            pos = np.cumsum(f[start:]) - 1  # position of each set block of w within the shard stream
            has = f[ids] == 1
            where = pos[ids[has] - start] + offs[w]
            res[has] = (res[has] + rv[where]).astype(np.float32)
        out[: k * B] = torch.from_numpy(res.reshape(-1))

    def scatter(self, packed, lst, k, dst):
        B = self.L.block_size
        if k:
            idx = _np(lst[:k]).astype(np.int64)
            d = dst.view(-1, B)
            d[torch.from_numpy(idx)] = packed[: k * B].view(-1, B)


class HostStagedComm:
    """gloo collectives for device tensors, staged through host memory (lets N processes share one GPU)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def all_gather_rows(self, out, inp):
        parts = [torch.empty_like(inp, device="cpu") for _ in range(self.world)]
        dist.all_gather(parts, inp.cpu(), group=self.group)
        out.copy_(torch.stack(parts).to(out.device))

    def exchange(self, sends, recvs):
        reqs, staged = [], []
        for p in range(self.world):
            if p == self.rank:
                continue
            if sends[p] is not None and sends[p].numel() > 0:
                reqs.append(dist.isend(sends[p].cpu(), p, group=self.group))
            if recvs[p] is not None and recvs[p].numel() > 0:
                buf = torch.empty(recvs[p].shape, dtype=recvs[p].dtype)
                reqs.append(dist.irecv(buf, p, group=self.group))
                staged.append((recvs[p], buf))
        for r in reqs:
            r.wait()
        for dst, buf in staged:
            dst.copy_(buf.to(dst.device))
