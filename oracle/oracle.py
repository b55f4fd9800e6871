"""numpy front end of liboracle.so — TEST INFRASTRUCTURE ONLY (see omr_oracle.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as
the checker / the timed CPU baseline.  It never backs the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_u32, _u64, _int, _vp, _dbl = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_double
_SIG = {
    "orc_sentinel": (_u32, [_u32, _u32]),
    "orc_gen_bitmap": (_u64, [_u32, _dbl, _u64, _vp]),
    "orc_fill": (None, [_vp, _u64, _u32, _int, _u32, _vp]),
    "orc_flags_from_data": (None, [_vp, _u64, _u32, _vp]),
    "orc_row_masks": (None, [_vp, _u64, _u32, _vp]),
    "orc_union_flags": (None, [_vp, _u32, _u64, _vp]),
    "orc_find_next_nonzero_block": (_u32, [_vp, _u32, _u32, _u32, _u32, _u32]),
    "orc_next_offsets": (None, [_vp, _u64, _u32, _u32, _u32, _vp]),
    "orc_block_sum": (None, [_vp, _u32, _u64, _u32, _u32, _u32, _vp, _vp]),
    "orc_lane_stream": (_u32, [_vp, _u64, _u32, _u32, _u32, _u32, _u32, _vp, _vp, _u32]),
    "orc_msg_simulate": (_int, [_vp, _vp, _u32, _u64, _u32, _u32, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "orc_cpu_baseline": (_dbl, [_vp, _vp, _u64, _u32, _u32, _u32, _u32, _u32, _int, _int, _vp, _vp, _vp]),
    "orc_cpu_baseline_cores": (_int, [_vp, _int]),
}
_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for k, (r, a) in _SIG.items():
            f = getattr(L, k)
            f.restype, f.argtypes = r, a
        _lib = L
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


def sentinel(B: int, NB: int) -> int:
    return lib().orc_sentinel(B, NB)


def gen_bitmap(worker_id: int, density: float, nb: int) -> np.ndarray:
    bm = np.empty(nb, dtype=np.int32)
    lib().orc_gen_bitmap(worker_id, density, nb, _p(bm))
    return bm


def fill(bitmap: np.ndarray, B: int, mode: int = 0, seed: int = 0) -> np.ndarray:
    buf = np.empty(bitmap.size * B, dtype=np.float32)
    lib().orc_fill(_p(bitmap), bitmap.size, B, mode, seed, _p(buf))
    return buf


def flags_from_data(buf: np.ndarray, B: int) -> np.ndarray:
    nb = buf.size // B
    f = np.empty(nb, dtype=np.int32)
    lib().orc_flags_from_data(_p(buf), nb, B, _p(f))
    return f


def row_masks(flags: np.ndarray, NB: int) -> np.ndarray:
    m = np.empty(flags.size // NB, dtype=np.uint64)
    lib().orc_row_masks(_p(flags), flags.size, NB, _p(m))
    return m


def union_flags(flags_list) -> np.ndarray:
    f = np.ascontiguousarray(np.stack(flags_list).astype(np.int32))
    out = np.empty(f.shape[1], dtype=np.int32)
    lib().orc_union_flags(_p(f), f.shape[0], f.shape[1], _p(out))
    return out


def find_next_nonzero_block(flags: np.ndarray, P: int, B: int, NB: int, tid: int, off: int) -> int:
    return lib().orc_find_next_nonzero_block(_p(flags), P, B, NB, tid, off)


def next_offsets(flags: np.ndarray, n: int, B: int, NB: int, parts: int) -> np.ndarray:
    nx = np.empty(n // B, dtype=np.uint32)
    lib().orc_next_offsets(_p(flags), n, B, NB, parts, _p(nx))
    return nx


def block_sum(bufs, n: int, B: int, NB: int, parts: int, uflags: np.ndarray, out: np.ndarray) -> np.ndarray:
    arr = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data for b in bufs])
    lib().orc_block_sum(arr, len(bufs), n, B, NB, parts, _p(uflags), _p(out))
    return out


def lane_stream(flags: np.ndarray, n: int, B: int, NB: int, parts: int, tid: int, bid: int):
    cap = (n // parts) // (B * NB) + 1
    cur = np.empty(cap, dtype=np.uint32)
    nxt = np.empty(cap, dtype=np.uint32)
    k = lib().orc_lane_stream(_p(flags), n, B, NB, parts, tid, bid, _p(cur), _p(nxt), cap)
    return cur[:k].copy(), nxt[:k].copy()


def cpu_baseline(x: np.ndarray, bitmap: np.ndarray, n: int, B: int, NB: int, parts: int, nthreads: int,
                 variant: int, warmups: int, rounds: int):
    """Mean seconds per round of the m=1 scan+aggregate (variant 0 reference-faithful bitmap walk,
    variant 1 data-derived fp32 scan), plus its outputs (flags, next, out)."""
    nb = n // B
    flags = np.zeros(nb, dtype=np.int32)
    nxt = np.zeros(nb, dtype=np.uint32)
    out = np.zeros(n, dtype=np.float32)
    t = lib().orc_cpu_baseline(_p(x), _p(bitmap), n, B, NB, parts, nthreads, variant, warmups, rounds,
                               _p(flags), _p(nxt), _p(out))
    if t < 0:
        raise ValueError("orc_cpu_baseline: nthreads must divide parts")
    return t, flags, nxt, out


def cpu_baseline_cores():
    """Core IDs the last cpu_baseline run pinned its threads to (empty for the single-thread path)."""
    buf = (ctypes.c_int * 256)()
    k = lib().orc_cpu_baseline_cores(buf, 256)
    return [int(buf[i]) for i in range(k)]


def msg_simulate(bufs, flags_list, n: int, B: int, NB: int, parts: int, rcap: int = 0, logs: bool = True):
    """Message-level round (the reference's per-slot state machines, client.cc:32-205 / server.cc:13-199, rank-order
    arrival).  Returns dict: outs (in-place results per worker), rounds [G], and with logs=True the wire logs
    wmsg [m][G][rcap][2048] f32, wimm [m][G][rcap], rmsg [G][rcap][2048], rimm [G][rcap]."""
    m = len(bufs)
    G = parts * 16
    if rcap <= 0:
        rcap = (n // parts) // (B * NB) + 2
    outs = [b.copy() for b in bufs]
    fl = [np.ascontiguousarray(f.astype(np.int32)) for f in flags_list]
    barr = (ctypes.c_void_p * m)(*[b.ctypes.data for b in bufs])
    farr = (ctypes.c_void_p * m)(*[f.ctypes.data for f in fl])
    oarr = (ctypes.c_void_p * m)(*[o.ctypes.data for o in outs])
    rounds = np.zeros(G, dtype=np.uint32)
    res = {"outs": outs, "rounds": rounds, "rcap": rcap}
    if logs:
        res["wmsg"] = np.zeros((m, G, rcap, 2048), dtype=np.float32)
        res["wimm"] = np.zeros((m, G, rcap), dtype=np.uint32)
        res["rmsg"] = np.zeros((G, rcap, 2048), dtype=np.float32)
        res["rimm"] = np.zeros((G, rcap), dtype=np.uint32)
        args = [_p(res["wmsg"]), _p(res["wimm"]), _p(res["rmsg"]), _p(res["rimm"])]
    else:
        args = [None, None, None, None]
    r = lib().orc_msg_simulate(barr, farr, m, n, B, NB, parts, rcap, *args, oarr, _p(rounds))
    if r < 0:
        raise ValueError("orc_msg_simulate: round capacity exceeded or inconsistent state")
    res["max_rounds"] = r
    return res
