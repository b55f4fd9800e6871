"""Generate the committed golden fixtures under tests/golden/ (run: python tests/golden/make_golden.py).

What the fixtures are: the reference holds no tests or vectors and cannot be built here,
so these are produced by the oracle (oracle/omr_oracle.c) from the reference's OWN generator — glibc
srand(myId+1)/rand() called exactly as client.cc:396-414 — and pinned by the reference's own known-answer
check (client.cc:449-465: the result equals the elementwise MPI_SUM of the inputs).  They freeze:
  flags_w     packed per-worker block flags (= the reference bitmaps, client.cc:406-414)
  next_w      per-worker next-offset arrays (find_next_nonzero_block(b*B + B*NB), client.cc:19-31)
  union_next  aggregator chain over the union (min_next, server.cc:86-96)
  counts      per-block number of contributing workers; with the 0.01f fill the summed block is the
              k-fold sequential fp32 sum of 0.01f (`ka_value[k]`), the CHECK known answer
  stream_*    one lane's worker send stream (client.cc:201-205, :87-102) as (current, next) pairs
Sizes are kept to KBs (compressed npz, loaded with allow_pickle=False).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle  # noqa: E402

# name: (n floats, block_size, density -r, m workers)
CONFIGS = {
    "c1_dense_4m_b256": (1 << 20, 256, 1.0, 1),             # BASELINE config 1
    "c2_scaled_8m_b256_r0095": (2 << 20, 256, 0.095, 1),    # config 2 shape, scaled
    "c3_scaled_16m_b1024_r00099": (4 << 20, 1024, 0.0099, 1),  # config 3 shape, scaled
    "m2_4m_b256_r0095": (1 << 20, 256, 0.095, 2),
    "m3_4m_b256_r03": (1 << 20, 256, 0.3, 3),
    "m4_8m_b1024_r00099": (2 << 20, 1024, 0.0099, 4),
    "m4_8m_b1024_r049": (2 << 20, 1024, 0.49, 4),
    "m8_4m_b512_r0095": (1 << 20, 512, 0.095, 8),
}
PARTS = 8


def ka_table(m: int) -> np.ndarray:
    """k-fold sequential fp32 sum of 0.01f starting from +0.0f, k = 0..m."""
    vals = [np.float32(0.0)]
    acc = np.float32(0.0)
    for _ in range(m):
        acc = np.float32(acc + np.float32(0.01))
        vals.append(acc)
    return np.array(vals, dtype=np.float32)


def make(name: str, n: int, B: int, r: float, m: int) -> dict:
    NB = 16 * 1024 // B
    nb = n // B
    flags = [oracle.gen_bitmap(w, r, nb) for w in range(m)]
    bufs = [oracle.fill(f, B) for f in flags]
    assert all((oracle.flags_from_data(b, B) == f).all() for b, f in zip(bufs, flags))
    nexts = [oracle.next_offsets(f, n, B, NB, PARTS) for f in flags]
    uf = oracle.union_flags(flags)
    unext = oracle.next_offsets(uf, n, B, NB, PARTS)
    out = np.zeros(n, dtype=np.float32)
    oracle.block_sum(bufs, n, B, NB, PARTS, uf, out)
    counts = np.sum(np.stack(flags), axis=0).astype(np.uint8)
    # known answer: every element of block b equals ka[counts[b]] (client.cc:449-465)
    ka = ka_table(m)
    assert (out.reshape(nb, B) == ka[counts][:, None]).all()
    cur, nxt = oracle.lane_stream(flags[0], n, B, NB, PARTS, tid=PARTS - 1, bid=NB - 1)
    meta = dict(name=name, n=n, block_size=B, num_lanes=NB, parts=PARTS, density=r, m=m,
                sentinel=oracle.sentinel(B, NB),
                nonzero=[int(f.sum()) for f in flags],
                sum_sha256=hashlib.sha256(out.tobytes()).hexdigest(),
                bitmap_sha256=[hashlib.sha256(f.tobytes()).hexdigest() for f in flags])
    arrays = dict(
        meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8),
        flags_w=np.stack([np.packbits(f.astype(np.uint8), bitorder="little") for f in flags]),
        next_w=np.stack(nexts),
        union_next=unext,
        counts=counts,
        ka_value=ka,
        stream_cur=cur,
        stream_next=nxt,
    )
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
    return meta


if __name__ == "__main__":
    oracle.build()
    for k, v in CONFIGS.items():
        meta = make(k, *v)
        print(k, meta["nonzero"], meta["sum_sha256"][:16])
