"""Oracle tests (CPU): the C restatement against the committed golden fixtures, an independent pure-Python
restatement of find_next_nonzero_block (client.cc:19-31), and the reference's own known-answer check
(client.cc:449-465).  The reference cannot be built here and has no vectors of its own: DESIGN.md §Oracle."""
import json
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
UINT32_MAX = 0xFFFFFFFF


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    return meta, z


GOLDEN_NAMES = sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith(".npz"))


def py_find_next_nonzero_block(bitmap, P, B, NB, tid, next_offset):
    """Line-by-line Python restatement of client.cc:19-31 with uint32 wrap-around."""
    off = next_offset & UINT32_MAX
    start = (P * tid) & UINT32_MAX
    bid = (off // B) % NB
    max_index = ((UINT32_MAX // B // NB - 1) * NB * B + bid * B) & UINT32_MAX
    while ((off - start) & UINT32_MAX) < P:
        if bitmap[off // B] == 1:
            return off
        off = (off + B * NB) & UINT32_MAX
    return max_index


@pytest.mark.parametrize("B,NB", [(256, 64), (512, 32), (1024, 16)])
def test_sentinel_value(B, NB):
    assert oracle.sentinel(B, NB) == 4294934528  # client.cc:24 for every MESSAGE_SIZE-derived NB


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_oracle_matches_golden(name):
    meta, z = load_golden(name)
    n, B, NB, P, m, r = meta["n"], meta["block_size"], meta["num_lanes"], meta["parts"], meta["m"], meta["density"]
    nb = n // B
    flags = [oracle.gen_bitmap(w, r, nb) for w in range(m)]
    for w in range(m):
        packed = np.packbits(flags[w].astype(np.uint8), bitorder="little")
        assert (packed == z["flags_w"][w]).all()
        assert int(flags[w].sum()) == meta["nonzero"][w]
        nxt = oracle.next_offsets(flags[w], n, B, NB, P)
        assert (nxt == z["next_w"][w]).all()
    uf = oracle.union_flags(flags)
    assert (oracle.next_offsets(uf, n, B, NB, P) == z["union_next"]).all()
    bufs = [oracle.fill(f, B) for f in flags]
    out = np.zeros(n, dtype=np.float32)
    oracle.block_sum(bufs, n, B, NB, P, uf, out)
    import hashlib
    assert hashlib.sha256(out.tobytes()).hexdigest() == meta["sum_sha256"]


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_known_answer_check(name):
    """client.cc:449-465: each worker's buffer after the round == MPI_SUM of the inputs, compared with !=."""
    meta, z = load_golden(name)
    n, B, NB, P, m, r = meta["n"], meta["block_size"], meta["num_lanes"], meta["parts"], meta["m"], meta["density"]
    nb = n // B
    flags = [oracle.gen_bitmap(w, r, nb) for w in range(m)]
    bufs = [oracle.fill(f, B) for f in flags]
    mpi_sum = np.zeros(n, dtype=np.float32)
    for b in bufs:  # MPI_Allreduce(input, output, DATA_SIZE, MPI_FLOAT, MPI_SUM) in rank order
        mpi_sum = (mpi_sum + b).astype(np.float32)
    uf = oracle.union_flags(flags)
    for w in range(m):  # in place on each worker's own buffer (client.cc:89)
        res = bufs[w].copy()
        oracle.block_sum(bufs, n, B, NB, P, uf, res)
        assert (res == mpi_sum).all()
    assert (mpi_sum.reshape(nb, B) == z["ka_value"][z["counts"]][:, None]).all()


@pytest.mark.parametrize("B,r,tid_list", [(256, 0.095, [0, 3, 7]), (1024, 0.0099, [0, 7]), (256, 0.0, [5])])
def test_find_next_matches_python_restatement(B, r, tid_list):
    NB = 16 * 1024 // B
    n = 1 << 20
    P = n // 8
    bm = oracle.gen_bitmap(1, r, n // B)
    rng = np.random.default_rng(0)
    for tid in tid_list:
        for _ in range(200):
            off = tid * P + int(rng.integers(0, P // B)) * B
            q = off + B * NB
            assert oracle.find_next_nonzero_block(bm, P, B, NB, tid, q) == \
                py_find_next_nonzero_block(bm, P, B, NB, tid, q)


def test_next_offsets_closed_form():
    """next[b] = first flagged block strictly after b in the same lane and partition, else SENT + bid*B."""
    n, B, NB, parts = 1 << 20, 256, 64, 8
    flags = oracle.gen_bitmap(2, 0.3, n // B)
    nxt = oracle.next_offsets(flags, n, B, NB, parts)
    rows_pp = n // parts // (B * NB)
    f = flags.reshape(parts, rows_pp, NB)
    sent = oracle.sentinel(B, NB)
    for p in range(parts):
        for lane in range(NB):
            following = sent + lane * B
            for row in range(rows_pp - 1, -1, -1):
                b = (p * rows_pp + row) * NB + lane
                assert nxt[b] == following
                if f[p, row, lane]:
                    following = b * B


def test_generator_density_mapping():
    """-r maps to ceil(101r)/100 of the blocks (client.cc:407): 0.095 -> 10 %, 0.1 -> 11 %, 0.0099 -> 1 %."""
    nb = 1 << 18
    for r, expect in [(0.095, 0.10), (0.1, 0.11), (0.0099, 0.01), (0.49, 0.50), (1.0, 1.0), (0.0, 0.0)]:
        frac = oracle.gen_bitmap(0, r, nb).mean()
        assert abs(frac - expect) < 0.005, (r, frac)


def test_worker_lane_stream():
    """Appendix A.3: a worker sends the lane head with next(head), then its own non-zero blocks in the lane,
    the last carrying the sentinel."""
    meta, z = load_golden("c2_scaled_8m_b256_r0095")
    n, B, NB, P = meta["n"], meta["block_size"], meta["num_lanes"], meta["parts"]
    flags = oracle.gen_bitmap(0, meta["density"], n // B)
    tid, bid = P - 1, NB - 1
    cur, nxt = oracle.lane_stream(flags, n, B, NB, P, tid, bid)
    assert (cur == z["stream_cur"]).all() and (nxt == z["stream_next"]).all()
    head = tid * (n // P) + bid * B
    own = [b * B for b in range(head // B + NB, (tid + 1) * (n // P) // B, NB) if flags[b]]
    assert list(cur) == [head] + own
    assert list(nxt[:-1]) == own and nxt[-1] == meta["sentinel"] + bid * B


def test_aggregator_min_next_is_union_chain():
    """server.cc:86-91: min over workers of their next offsets == next over the union flags."""
    meta, z = load_golden("m4_8m_b1024_r049")
    mins = np.min(z["next_w"], axis=0)
    assert (mins == z["union_next"]).all()


def test_cpu_baseline_variants_agree():
    n, B, NB, parts = 1 << 20, 256, 64, 8
    bm = oracle.gen_bitmap(0, 0.095, n // B)
    x = oracle.fill(bm, B)
    t1, f1, nx1, out1 = oracle.cpu_baseline(x, bm, n, B, NB, parts, 8, 1, 0, 2)
    t0, _, nx0, out0 = oracle.cpu_baseline(x, bm, n, B, NB, parts, 8, 0, 0, 2)
    t1s, f1s, nx1s, out1s = oracle.cpu_baseline(x, bm, n, B, NB, parts, 1, 1, 0, 1)
    assert (f1 == bm).all() and (f1s == bm).all()
    assert (out0 == out1).all() and (out1s == out1).all()
    ref = oracle.next_offsets(bm, n, B, NB, parts)
    assert (nx1 == ref).all() and (nx1s == ref).all()
    visited = (bm == 1)
    rows_pp = n // B // NB // parts
    heads = ((np.arange(n // B) // NB) % rows_pp) == 0
    sel = visited | heads
    assert (nx0[sel] == ref[sel]).all()
    assert t0 > 0 and t1 > 0


# ------------------------------------------------------------------ message-level state machines (orc_msg_simulate)

@pytest.mark.parametrize("n,B,m,density", [(1 << 20, 256, 1, 0.095), (1 << 20, 256, 3, 0.3), (2 << 20, 512, 2, 0.1),
                                           (4 << 20, 1024, 4, 0.2), (1 << 20, 256, 2, 1.0), (1 << 20, 256, 2, 0.0)])
def test_msg_simulate_known_answer_and_wire_invariants(n, B, m, density):
    """The literal per-slot state machines (client.cc:32-205, server.cc:13-199) end every worker on the dense
    rank-order sum (the reference's CHECK, client.cc:449-465), and their wire traffic has the shape SURVEY.md
    Appendix A states: imm = (len << 16) | gs, replies carry the union chain (server.cc:86-96 min_next), worker
    messages carry the worker's own non-zero blocks with its own next offsets (after the lane heads)."""
    NB, P = 16384 // B, 8
    BPM = 1024 // B
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, n // B), B, mode=1, seed=w + 2) for w in range(m)]
    flags = [oracle.flags_from_data(b, B) for b in bufs]
    ref = oracle.msg_simulate(bufs, flags, n, B, NB, P)
    uf = oracle.union_flags(flags)
    unext = oracle.next_offsets(uf, n, B, NB, P)
    own_next = [oracle.next_offsets(f, n, B, NB, P) for f in flags]
    for w in range(m):
        exp = bufs[w].copy()
        oracle.block_sum(bufs, n, B, NB, P, uf, exp)
        assert (ref["outs"][w].view(np.uint32) == exp.view(np.uint32)).all()
    sent = oracle.sentinel(B, NB)
    for gs in range(P * 16):
        R = int(ref["rounds"][gs])
        assert R >= 1
        cur = {}  # lane -> the block its round carries
        t, s = divmod(gs, 16)
        for j in range(BPM):
            cur[s * BPM + j] = (t * (n // P)) // B + s * BPM + j
        for r in range(R):
            rimm = int(ref["rimm"][gs, r])
            ln = rimm >> 16
            assert rimm & 0xFFFF == gs and 1 <= ln <= BPM
            meta = ref["rmsg"][gs, r, ln * B: ln * B + ln].view(np.uint32)
            assert sorted((int(x) // B) % NB for x in meta) == sorted(cur), "reply lanes = the active lanes"
            for w in range(m):
                wi = int(ref["wimm"][w, gs, r])
                if wi == 0:
                    continue
                lw = wi >> 16
                assert wi & 0xFFFF == gs
                wmeta = ref["wmsg"][w, gs, r, lw * B: lw * B + lw].view(np.uint32)
                for k, nx in enumerate(wmeta):
                    lane = (int(nx) // B) % NB
                    b = cur[lane]
                    assert r == 0 or flags[w][b] == 1, "after the heads a worker sends only its non-zero blocks"
                    assert int(nx) == int(own_next[w][b]), "each block travels with the worker's own next offset"
                    blk = ref["wmsg"][w, gs, r, k * B:(k + 1) * B]
                    assert (blk.view(np.uint32) == bufs[w][b * B:(b + 1) * B].view(np.uint32)).all()
            nxt = {}
            for x in meta:
                lane = (int(x) // B) % NB
                assert int(x) == int(unext[cur[lane]]), "min_next = the union chain"
                if int(x) < sent:
                    nxt[lane] = int(x) // B
            cur = nxt
        assert not cur, "a slot ends when every lane reaches its sentinel"
