"""The round's stream layouts in one process, in the order that once failed, and the side streams'
hardware-queue check (round 6, omr_ar_plan_queue_report).

`gpurun_out/r05b/inproc_nogroup.log` recorded `hipEventRecord: invalid resource handle` on the first round of the N > 1
layout after one-launch rounds on the null and on a created stream, then a re-plan (tools/round_inproc_r05.py).  That
run was of an uncommitted working tree (its files predate the next commit, 8e2904c); every later run of the same
sequence passed.  This test runs the sequence itself -- one-launch world-1 rounds (solo), the multi-rank round's path at
world 1 with two side streams (general) and with one (general1), each on the null stream and on a stream created for
it, deferred rounds over four rotating inputs, re-planned between layouts -- and checks every output against the
oracle (rank-order sums, server.cc:97-98, in place of client.cc:89's copy), so a destroyed stream or event still in use
across a re-plan fails here by name."""
import numpy as np
import pytest
import torch

import oracle
from omr import Layout, cdist

pytestmark = pytest.mark.gpu
B = 256


def _inputs(L, gpu, k=4, density=0.1):
    xs, exps = [], []
    for i in range(k):
        x = oracle.fill(oracle.gen_bitmap(i, density, L.nb), B, mode=1, seed=20 + i)
        f = oracle.flags_from_data(x, B)
        exp = x.copy()
        oracle.block_sum([x], L.n, B, L.num_lanes, 8, f, exp)
        xs.append(torch.from_numpy(x).to(gpu))
        exps.append(exp)
    return xs, exps


def _rounds(eng, xs, exps, st, thread, rounds=14):
    """Deferred rounds on stream st (reduce-scatter and all-reduce alternating in pairs), joined, every output checked."""
    with torch.cuda.stream(st):
        outs = [x.clone() for x in xs]
        for k in range(rounds):
            i = k % len(xs)
            eng.run(xs[i], out=outs[i], mode=(k // 4) % 2, async_=True, defer=True, thread=thread, counts=False)
        eng.join(st)
    st.synchronize()
    for i, (o, e) in enumerate(zip(outs, exps)):
        assert (o.cpu().numpy().view(np.uint32) == e.view(np.uint32)).all(), i


@pytest.mark.parametrize("pipe", ["defer", "thread"])
def test_layout_sequence_matches_oracle(gpu, pipe):
    L = Layout(n=1 << 22, block_size=B)
    xs, exps = _inputs(L, gpu)
    eng = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        for layout in ("solo", "general", "general1"):
            eng.test_world1_round(layout != "solo")
            eng.replan()  # (the hook applies to plans made after it)
            if layout == "general1":
                eng.set_side_streams(1)
            for sname in ("null", "created"):
                st = torch.cuda.current_stream(gpu) if sname == "null" else torch.cuda.Stream(gpu)
                _rounds(eng, xs, exps, st, thread=pipe == "thread")
                rep = eng.queue_report()
                if layout == "solo":  # the one-launch round has no side stream: nothing to check
                    assert rep["probes"] == 0, rep
                else:
                    assert rep["disjoint"] in (0, 1) and rep["probes"] >= (3 if layout == "general" else 1), rep
    finally:
        assert eng.close() == (0, 0)


def test_queue_check_keeps_side_streams_apart(gpu):
    """On a stream created after the plan (the cell round 5 measured at 69.5-75.6 us per round), the checked side
    streams end on queues of their own: a probe of each against the caller's stream, and of the two against each other,
    lets its mark run while the other's queue is held.  The same rounds with the check off stay bit-exact."""
    L = Layout(n=1 << 22, block_size=B)
    xs, exps = _inputs(L, gpu, k=4, density=0.3)
    eng = cdist.CppSparseAllreduce(L, gpu, transport="rccl1")
    try:
        eng.test_world1_round(True)
        eng.replan()
        created = torch.cuda.Stream(gpu)
        _rounds(eng, xs, exps, created, thread=False)
        rep = eng.queue_report()
        assert rep["probes"] >= 3, rep
        assert rep["disjoint"] == 1, rep  # 4 hardware queues: the caller's + two side streams fit
        eng.set_queue_check(False)
        _rounds(eng, xs, exps, torch.cuda.Stream(gpu), thread=False)
        assert eng.queue_report()["probes"] == rep["probes"]  # (no probe with the check off)
    finally:
        assert eng.close() == (0, 0)
