"""ctypes binding of the C ABI in include/omr.h (libomr.so, built in-tree for gfx950).

The library is the product: there is no CPU fallback.  If libomr.so is missing or fails to load, every
entry point raises — a GPU run that silently fell back to another implementation would void the parity
claims.  torch is imported first on purpose: torch's ROCm wheel ships its own libamdhip64.so.7, and the
dynamic loader must bind libomr.so to that same HIP runtime (same soname) rather than load a second one.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libomr.so")

c_u32 = ctypes.c_uint32
c_u64 = ctypes.c_uint64
c_int = ctypes.c_int
c_vp = ctypes.c_void_p
c_dbl = ctypes.c_double
c_size = ctypes.c_size_t

OMR_EINVAL = -1
OMR_MAX_WORKERS = 16

# name -> (restype, argtypes); mirrors include/omr.h one-to-one
SIGNATURES = {
    "omr_abi_version": (c_int, []),
    "omr_last_error": (ctypes.c_char_p, []),
    "omr_num_lanes": (c_u32, [c_u32]),
    "omr_sentinel": (c_u32, [c_u32, c_u32]),
    "omr_layout_check": (c_int, [c_u64, c_u32, c_u32, c_u32]),
    "omr_gen_bitmap": (c_int, [c_u32, c_dbl, c_u64, c_vp, c_vp]),
    "omr_fill_blocks_f32": (c_int, [c_vp, c_u64, c_u32, c_int, c_u32, c_vp, c_vp]),
    "omr_scan_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp]),
    "omr_scan_sum_f32": (c_int, [c_vp, c_u32, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "omr_scan_workspace_bytes": (c_size, [c_u64, c_u32, c_u32, c_u32]),
    "omr_scan_sum_fused_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "omr_scan_partition_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_size,
                                       c_vp]),
    "omr_scan_sum_rows_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_u64, c_u64, c_vp, c_vp, c_vp, c_vp]),
    "omr_next_offsets": (c_int, [c_vp, c_u32, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp]),
    "omr_block_sum_f32": (c_int, [c_vp, c_u32, c_vp, c_u32, c_u32, c_vp, c_vp]),
    "omr_dense_sum_f32": (c_int, [c_vp, c_u32, c_u64, c_vp, c_vp]),
    "omr_compact_workspace_bytes": (c_size, [c_u64]),
    "omr_compact": (c_int, [c_vp, c_u64, c_u64, c_u32, c_vp, c_vp, c_vp, c_size, c_vp]),
    "omr_gather_blocks_f32": (c_int, [c_vp, c_vp, c_u32, c_u32, c_vp, c_vp]),
    "omr_scatter_blocks_f32": (c_int, [c_vp, c_vp, c_u32, c_u32, c_vp, c_vp]),
    "omr_mask_union": (c_int, [c_vp, c_u32, c_u64, c_u32, c_u32, c_int, c_vp, c_vp]),
    "omr_prefix_workspace_bytes": (c_size, [c_u64, c_u32]),
    "omr_row_prefix": (c_int, [c_vp, c_u32, c_u64, c_vp, c_vp, c_size, c_vp]),
    "omr_worker_scan_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "omr_round_plan": (c_int, [c_vp, c_u32, c_u64, c_u32, c_u32, c_vp, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_u32, c_vp]),
    "omr_round_plan_workspace_words": (c_u64, []),
    "omr_move_blocks_f32": (c_int, [c_vp, c_vp, c_int, c_vp, c_vp, c_u64, c_u32, c_u32, c_u64, c_u64, c_vp]),
    "omr_shard_sum_f32": (c_int, [c_vp, c_u32, c_vp, c_vp, c_vp, c_u32, c_vp, c_vp, c_u64, c_u64, c_u64, c_u32,
                                  c_u32, c_int, c_vp, c_vp]),
    "omr_worker_scan_pack_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32,
                                         ctypes.c_int32, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "omr_pack_geometry": (c_int, [c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp]),
    "omr_pack_supported": (c_int, [c_u64, c_u32, c_u32, c_u32, c_vp, c_u32]),
    "omr_pack_send_offset": (c_u64, [c_vp, c_u32, ctypes.c_int32, c_u32, c_u32, c_u32, c_vp]),
    "omr_worker_scan_tally_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32,
                                          c_vp, c_size, c_vp]),
    "omr_tally_publish": (c_int, [c_vp, c_u32, c_vp, c_u32, c_vp]),
    "omr_tally_slots": (c_u32, [c_u64, c_u32, c_u32, c_u32]),
    "omr_round_plan_list": (c_int, [c_vp, c_u32, c_u64, c_u64, c_u32, c_u32, c_vp, c_u32, c_vp, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_u32, c_vp, c_u32, c_vp, c_u32, c_vp, c_vp]),
    "omr_round_check_slots": (c_u32, [c_u64, c_u32, c_u32, c_u32]),
    "omr_shard_sum_stride_f32": (c_int, [c_vp, c_u32, c_vp, c_vp, c_vp, c_u64, c_u32, c_vp, c_vp, c_u64, c_u64, c_u64,
                                         c_u32, c_u32, c_int, c_vp, c_vp]),
    "omr_worker_scan_check_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_size,
                                          c_vp, c_u32, c_vp, c_vp]),
    "omr_worker_scan_pack_check_f32": (c_int, [c_vp, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_u32,
                                               ctypes.c_int32, c_vp, c_vp, c_vp, c_vp, c_size, c_vp, c_u32, c_vp,
                                               c_vp]),
    "omr_round_plan_check": (c_int, [c_vp, c_u32, c_u64, c_u64, c_u32, c_u32, c_vp, c_u32, c_vp, c_vp, c_vp, c_vp,
                                     c_vp, c_vp, c_u32, c_vp, c_u32, c_vp, c_u32, c_vp, c_u64, c_u32, c_vp, c_vp]),
    "omr_sum_list_geometry": (c_int, [c_u64, c_u32, c_u32, c_u32, c_u64, c_u64, c_u32, c_vp, c_vp]),
    "omr_sum_list_build": (c_int, [c_vp, c_u32, c_u64, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp]),
    "omr_shard_sum_list_f32": (c_int, [c_vp, c_vp, c_vp, c_u32, c_u64, c_u32, c_u32, c_u32, c_vp, c_vp, c_int, c_vp,
                                       c_vp]),
    "omr_msg_plan_create": (c_int, [c_u64, c_u32, c_u32, c_u32, c_u32, c_vp]),
    "omr_msg_plan_destroy": (c_int, [c_vp]),
    "omr_msg_round_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "omr_msg_logs": (c_int, [c_vp, c_u32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "omr_msg_sched_bytes": (c_size, []),
    "omr_msg_schedule": (c_int, [c_vp, c_u32, c_vp, c_u64, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp, c_vp]),
    "omr_msg_pack_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_vp, c_vp, c_vp]),
    "omr_msg_aggregate_f32": (c_int, [c_vp, c_vp, c_u32, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_u32, c_u32,
                                      c_vp, c_vp, c_vp]),
    "omr_msg_unpack_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_u32, c_u32, c_u32, c_u32, c_vp, c_vp]),
    "omr_sparse_block_sum_f32": (c_int, [c_vp, c_vp, c_vp, c_u32, c_u64, c_vp, c_u64, c_u32, c_vp, c_u32, c_u32,
                                         c_vp, c_vp]),
    "omr_host_last_error": (ctypes.c_char_p, []),
    "omr_host_register": (c_int, [c_vp, c_size]),
    "omr_host_unregister": (c_int, [c_vp]),
    "omr_host_plan_create": (c_int, [c_u64, c_u32, c_u32, c_u32, c_u64, c_vp]),
    "omr_host_plan_destroy": (c_int, [c_vp]),
    "omr_host_scan_sum_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
    "omr_host_scan_sum_zero_copy_f32": (c_int, [c_vp, c_vp, c_vp, c_vp, c_vp]),
}

_lib = None


class SumList(ctypes.Structure):
    """struct omr_sum_list (include/omr.h): an aggregator's shard-sum pair list."""
    _fields_ = [("records", c_vp), ("counts", c_vp), ("row_begin", c_u64), ("row_end", c_u64),
                ("pos_offset", c_u64), ("me", ctypes.c_uint32), ("recv_offsets", c_u64 * OMR_MAX_WORKERS)]


class OmrError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load libomr.so once; raise OmrError (never fall back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("OMR_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise OmrError(f"libomr.so not found at {p}: build it with __graft_entry__.build() "
                       f"or `make -C omnireduce-rdma-demo_amd` (no CPU fallback exists)")
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.omr_abi_version() != 2:
        raise OmrError(f"libomr ABI {lib.omr_abi_version()} != 2 (rebuild: make -C omnireduce-rdma-demo_amd)")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().omr_last_error().decode(errors="replace")
        raise OmrError(f"{what} failed (rc={rc}): {msg}")
