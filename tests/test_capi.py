"""C-ABI tests that need no GPU: the library loads, exports every symbol include/omr.h declares, and its
host-only logic (layout validation, sentinel, the reference generator restatement) is right."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from omr import _lib, Layout
from omr import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "omr.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(omr_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.omr_abi_version() == 2


@pytest.mark.parametrize("B,NB", [(256, 64), (512, 32), (1024, 16)])
def test_num_lanes_and_sentinel(B, NB):
    lib = _lib.load()
    assert lib.omr_num_lanes(B) == NB  # common.h:36-37
    assert lib.omr_sentinel(B, NB) == 4294934528 == Layout(n=8 * NB * B, block_size=B).sentinel


def test_layout_check_rejects_bad_layouts():
    lib = _lib.load()
    assert lib.omr_layout_check(1 << 20, 256, 64, 8) == 0
    assert lib.omr_layout_check(64 << 20, 256, 64, 8) == 0
    assert lib.omr_layout_check(256 << 20, 1024, 16, 8) == 0
    assert lib.omr_layout_check(1 << 30, 256, 64, 8) == 0  # config 5: 4 GiB per rank
    assert lib.omr_layout_check(1 << 20, 128, 128, 8) == _lib.OMR_EINVAL  # NB > 64 unsupported
    assert b"block_size" in lib.omr_last_error()
    assert lib.omr_layout_check((1 << 20) + 256, 256, 64, 8) == _lib.OMR_EINVAL  # ragged partition
    assert lib.omr_layout_check(0, 256, 64, 8) == _lib.OMR_EINVAL
    assert lib.omr_layout_check(1 << 32, 256, 64, 8) == _lib.OMR_EINVAL  # past the uint32 sentinel


def test_entry_points_validate_before_launching():
    """Argument errors return OMR_EINVAL without touching the device (safe on a GPU-less host)."""
    lib = _lib.load()
    assert lib.omr_scan_f32(None, 1 << 20, 300, 64, 8, None, None, None, None) == _lib.OMR_EINVAL
    assert lib.omr_scan_sum_f32(None, 0, 1 << 20, 256, 64, 8, None, None, None, None, None) == _lib.OMR_EINVAL
    assert lib.omr_block_sum_f32(None, 1, None, 4, 100, None, None) == _lib.OMR_EINVAL
    assert lib.omr_block_sum_f32(None, 1, None, 0, 256, None, None) == 0  # empty list is a no-op
    assert lib.omr_compact(None, 5, 3, 64, None, None, None, 0, None) == _lib.OMR_EINVAL
    assert lib.omr_fill_blocks_f32(None, 4, 256, 7, 0, None, None) == _lib.OMR_EINVAL
    assert lib.omr_dense_sum_f32(None, 0, 16, None, None) == _lib.OMR_EINVAL  # m out of range
    assert lib.omr_dense_sum_f32(None, 2, 6, None, None) == _lib.OMR_EINVAL  # n not a multiple of 4
    assert lib.omr_dense_sum_f32(None, 2, 0, None, None) == 0  # empty is a no-op


@pytest.mark.parametrize("wid", [0, 1, 2, 7])
@pytest.mark.parametrize("r", [0.095, 0.0099, 0.49, 1.0, 0.3])
def test_product_generator_equals_glibc(wid, r):
    """omr_gen_bitmap restates glibc rand(); the oracle calls glibc srand/rand as client.cc:396-414 does."""
    nb = 20000
    assert (ops.gen_bitmap(wid, r, nb) == oracle.gen_bitmap(wid, r, nb)).all()


def test_product_generator_count():
    lib = _lib.load()
    bm = np.empty(4096, dtype=np.int32)
    cnt = ctypes.c_uint64()
    assert lib.omr_gen_bitmap(0, 0.095, 4096, bm.ctypes.data_as(ctypes.c_void_p), ctypes.byref(cnt)) == 0
    assert cnt.value == int(bm.sum())


def test_layout_class():
    L = Layout.from_bytes(256 << 20, 256)
    assert (L.n, L.num_lanes, L.nb, L.rows, L.rows_per_part) == (64 << 20, 64, 262144, 4096, 512)
    L3 = Layout.from_bytes(1 << 30, 1024)
    assert (L3.num_lanes, L3.rows_per_part, L3.blocks_per_message) == (16, 2048, 1)
    assert L.lane_of(L.head_offset(3, 17)) == 17 and L.partition_of(L.head_offset(3, 17)) == 3
    assert L.global_slot(2, 5) == 37
    with pytest.raises(ValueError):
        Layout(n=(1 << 20) + 256)


def test_dist_library_exports_every_declared_symbol():
    """libomr_dist.so (the multi-rank round, include/omr_dist.h) loads without a GPU and exports what its header
    declares; the ctypes binding (omr/cdist.py) binds every one of them."""
    import inspect
    from omr import cdist
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "omr_dist.h")).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(omr_[a-z0-9_]+)\s*\(", src)))
    lib = cdist.load()
    for name in declared:
        assert hasattr(lib, name), name
    bound = set(re.findall(r'"(omr_[a-z0-9_]+)"', inspect.getsource(cdist.load)))
    assert sorted(set(declared) - bound) == [], "omr_dist.h entry points without a ctypes binding"


@pytest.mark.parametrize("mib,B,S,gps,entries", [(256, 256, 512, 8, 4096), (256, 1024, 256, 4, 1024),
                                                 (8, 256, 16, 1, 512)])
def test_pack_geometry(mib, B, S, gps, entries):
    """The fused pack's column segments and position table (host-only logic of omr_pack_geometry): config 4's
    256 MiB at B=256 scans one 512-row segment per (partition, lane) column; B=1024 has two per column."""
    lib = _lib.load()
    L = Layout.from_bytes(mib << 20, B)
    s, g, e = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    assert lib.omr_pack_geometry(L.n, B, L.num_lanes, L.num_threads, ctypes.byref(s), ctypes.byref(g),
                                 ctypes.byref(e)) == 0
    assert (s.value, g.value, e.value) == (S, gps, entries)


@pytest.mark.parametrize("world", range(1, 9))
def test_pack_supported_worlds(world):
    """Shards must be whole column segments: worlds 1, 2, 4, 8 of config 4 pack in the scan; 3, 5, 6, 7 (ragged
    shards) keep the separate pack pass."""
    lib = _lib.load()
    L = Layout.from_bytes(256 << 20, 256)
    b = np.array([s * L.rows // world for s in range(world + 1)], dtype=np.uint64)
    rc = lib.omr_pack_supported(L.n, 256, L.num_lanes, L.num_threads, b.ctypes.data_as(ctypes.c_void_p), world)
    assert (rc == 0) == (world in (1, 2, 4, 8)), (world, rc)


@pytest.mark.parametrize("world,own", [(8, 3), (4, 0), (2, 1), (8, -1), (3, 2)])
def test_pack_send_offset(world, own):
    """Round 5's compact send buffer (omr_pack_send_offset, host-only): the other shards' streams back to back in shard
    order, the own shard left out; the buffer's size is the tensor less the own shard."""
    lib = _lib.load()
    L = Layout.from_bytes(256 << 20, 256)
    b = np.array([s * L.rows // world for s in range(world + 1)], dtype=np.uint64)
    rowf = L.num_lanes * 256
    total = ctypes.c_uint64()
    at = 0
    for s in range(world):
        off = lib.omr_pack_send_offset(b.ctypes.data_as(ctypes.c_void_p), world, own, s, L.num_lanes, 256,
                                       ctypes.byref(total))
        if s == own:
            continue
        assert off == at * rowf, (s, off, at)
        at += int(b[s + 1] - b[s])
    own_rows = int(b[own + 1] - b[own]) if own >= 0 else 0
    assert total.value == (L.rows - own_rows) * rowf


def test_round_plan_workspace_and_validation():
    """The row-chunk plan's workspace size (one ticket word + 64 chunks x 17 tagged totals + the round check's 17
    tagged findings), and its argument checks,
    which return before any launch: seq 0 (a zero-filled word carries it), count 0, a NULL workspace."""
    lib = _lib.load()
    assert lib.omr_round_plan_workspace_words() == 1 + 64 * 17 + 17
    fake = ctypes.c_void_p(0x1000)  # (never dereferenced: the checks come first)
    args = lambda count, ws, seq: (fake, count, 4096, 512, 64, fake, 9, fake, None, fake, fake, None, ws, seq, None)  # noqa: E731
    assert lib.omr_round_plan(*args(8, fake, 0)) == _lib.OMR_EINVAL
    assert b"seq 0" in lib.omr_last_error()
    assert lib.omr_round_plan(*args(0, fake, 1)) == _lib.OMR_EINVAL
    assert lib.omr_round_plan(*args(8, None, 1)) == _lib.OMR_EINVAL


@pytest.mark.parametrize("mib,B", [(256, 256), (1024, 1024), (4, 256)])
def test_tally_slots(mib, B):
    """The one-rank round's tally: one slot per workgroup of its launch, (partition, lane) columns x segments."""
    lib = _lib.load()
    L = Layout.from_bytes(mib << 20, B)
    s, g, e = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    assert lib.omr_pack_geometry(L.n, B, L.num_lanes, L.num_threads, ctypes.byref(s), ctypes.byref(g),
                                 ctypes.byref(e)) == 0
    segments = L.rows_per_part // s.value
    assert lib.omr_tally_slots(L.n, B, L.num_lanes, L.num_threads) == L.num_threads * L.num_lanes * segments
