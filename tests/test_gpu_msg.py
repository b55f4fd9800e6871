"""GPU parity of the message-level round (include/omr.h omr_msg_*): every worker message and aggregator reply in
the reference's wire format (common.cc:399-443) against the oracle's literal restatement of the two per-slot state
machines (client.cc:32-205, server.cc:13-199; oracle/omr_oracle.c orc_msg_simulate), rank-order arrival.
Bar: bit-exact — round counts, imm words, every payload byte of every valid message (blocks and next offsets),
and the in-place results (which also equal the reference's own known answer, the dense rank-order sum)."""
import numpy as np
import pytest
import torch

import oracle
from omr import Layout, ops

pytestmark = pytest.mark.gpu


def check_against_oracle(bufs_np, L):
    dev = torch.device("cuda:0")
    m = len(bufs_np)
    B, NB, P = L.block_size, L.num_lanes, L.num_threads
    flags = [oracle.flags_from_data(b, B) for b in bufs_np]
    ref = oracle.msg_simulate(bufs_np, flags, L.n, B, NB, P)
    bufs = [torch.from_numpy(b).to(dev) for b in bufs_np]
    outs = [b.clone() for b in bufs]
    eng = ops.MessageRound(L, m, device=dev)
    maxr = eng.run(bufs, outs)
    torch.cuda.synchronize()
    assert maxr == ref["max_rounds"]
    G = P * 16
    for w in range(m):
        lg = eng.logs(w)
        rounds = lg["rounds"].cpu().numpy().astype(np.int64)
        assert (rounds == ref["rounds"].astype(np.int64)).all(), "rounds per slot"
        imm = lg["imm"].cpu().numpy().view(np.uint32)
        rimm = lg["reply_imm"].cpu().numpy().view(np.uint32)
        msgs = lg["messages"].cpu().numpy()
        reps = lg["replies"].cpu().numpy()
        for gs in range(G):
            R = int(rounds[gs])
            assert (imm[gs, :R] == ref["wimm"][w, gs, :R]).all(), f"worker {w} imm, slot {gs}"
            assert (rimm[gs, :R] == ref["rimm"][gs, :R]).all(), f"reply imm, slot {gs}"
            for r in range(R):
                ln = int(imm[gs, r] >> 16)
                words = ln * B + ln
                assert (msgs[gs, r, :words].view(np.uint32) == ref["wmsg"][w, gs, r, :words].view(np.uint32)).all(), \
                    f"worker {w} message slot {gs} round {r}"
                lr = int(rimm[gs, r] >> 16)
                words = lr * B + lr
                assert (reps[gs, r, :words].view(np.uint32) == ref["rmsg"][gs, r, :words].view(np.uint32)).all(), \
                    f"reply slot {gs} round {r}"
        assert (outs[w].cpu().numpy().view(np.uint32) == ref["outs"][w].view(np.uint32)).all(), f"worker {w} result"
    # the reference's own known answer (client.cc:449-465, done right): every worker holds the rank-order sum
    uf = oracle.union_flags(flags)
    for w in range(m):
        exp = bufs_np[w].copy()
        oracle.block_sum(bufs_np, L.n, B, NB, P, uf, exp)
        assert (outs[w].cpu().numpy().view(np.uint32) == exp.view(np.uint32)).all()
    eng.close()


@pytest.mark.parametrize("n,B,m,density,mode", [
    (1 << 20, 256, 1, 0.095, 0),     # config 1 layout, reference fill
    (1 << 20, 256, 2, 0.3, 1),
    (1 << 20, 256, 3, 0.095, 1),
    (4 << 20, 256, 4, 0.05, 1),      # longer chains: many protocol rounds, reply orders diverge
    (4 << 20, 256, 8, 0.2, 1),
    (2 << 20, 512, 3, 0.3, 1),       # BLOCKS_PER_MESSAGE = 2
    (4 << 20, 1024, 3, 0.1, 1),      # BLOCKS_PER_MESSAGE = 1
    (1 << 20, 256, 2, 1.0, 1),       # dense
    (1 << 20, 256, 2, 0.0, 1),       # all zero: only the lane heads travel
])
def test_msg_round_matches_state_machines(gpu, n, B, m, density, mode):
    L = Layout(n=n, block_size=B)
    bufs = [oracle.fill(oracle.gen_bitmap(w, density, L.nb), B, mode=mode, seed=w + 1) for w in range(m)]
    check_against_oracle(bufs, L)


def test_msg_round_in_place_twice(gpu):
    """In place (outs = bufs, client.cc:89), run twice: the second round starts from the first's sums."""
    L = Layout(n=1 << 20)
    m = 3
    bufs_np = [oracle.fill(oracle.gen_bitmap(w, 0.2, L.nb), L.block_size, mode=1, seed=w) for w in range(m)]
    dev = torch.device("cuda:0")
    bufs = [torch.from_numpy(b.copy()).to(dev) for b in bufs_np]
    eng = ops.MessageRound(L, m, device=dev)
    cur = [b.copy() for b in bufs_np]
    for _ in range(2):
        eng.run(bufs)
        fl = [oracle.flags_from_data(c, L.block_size) for c in cur]
        ref = oracle.msg_simulate(cur, fl, L.n, L.block_size, L.num_lanes, L.num_threads, logs=False)
        cur = ref["outs"]
        for w in range(m):
            assert (bufs[w].cpu().numpy().view(np.uint32) == cur[w].view(np.uint32)).all()
    eng.close()
