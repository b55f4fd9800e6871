#!/usr/bin/env python3
"""bench.py — device-resident block scan+sum throughput (BASELINE.json metric), one JSON line on rank 0.

Workload at N=1 (BASELINE.json configs[1]): a 256 MiB fp32 gradient, BLOCK_SIZE=256 (64 lanes, 8 partitions),
reference generator at -r 0.095 (10 % of blocks non-zero = 90 % block-sparse), one worker, already resident
in HBM.  One step = one pass of the hot path over it: one launch of the single-pass kernel k_scan1f (per-block
flags, next offsets, and the aggregated non-zero blocks written back in place, as client.cc:89 does).
(0.0f + x == x for the generator's data, so every step sees the same input.)  Four input buffer sets are rotated
so that no step re-reads data the 256 MiB Infinity Cache still holds from the previous use.
N>1 (torch.distributed.run, one rank per GPU): each rank is worker r with its own 256 MiB tensor (seed r+1) and
aggregator for shard r; a step is one OmniReduce round driven from C++ (libomr_dist.so over RCCL): worker scan,
row-mask all-gather, round plan, pack, grouped send/recv of the non-zero blocks over xGMI, rank-order shard sums
(reduce-scatter, BASELINE config 4; --dist-mode allreduce also returns every shard's sums to every worker).
value   = bytes of gradient processed by all ranks per second (decimal GB/s, logical tensor bytes; the
          reference's "alg bw" divides the same quantity by 2^30: client.cc:445)
roofline= the dominant kernel (k_scan1f) timed with HIP events on its own stream inside the timed region;
          achieved = its algorithmic bytes per launch / its mean duration
cpu_baseline = the oracle's C restatement of the reference loop (client.cc:19-31 + server.cc:83-99) on this
          host, 8 pthreads one per partition as client.cc:384-392, rank 0 at N=1 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "omnireduce-rdma-demo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from omr import Layout, ops  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBPS = 153.0  # one of a GPU's 7 point-to-point xGMI links (the task's hardware notes; not in the guide)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs of this node, one rank each (default 1).  N > 1 without a launcher: bench.py starts "
                        "torch.distributed.run with N ranks as a child process and relays rank 0's line; it exits "
                        "non-zero when the node has fewer than N GPUs")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--size-mib", type=int, default=256)
    p.add_argument("--block-size", type=int, default=256)
    p.add_argument("--density", type=float, default=0.095, help="reference -r (0.095 -> 10%% non-zero)")
    p.add_argument("--workers", type=int, default=1, help="m worker tensors per GPU (N=1 only)")
    p.add_argument("--rotate", type=int, default=4, help="buffer sets rotated to defeat the Infinity Cache")
    p.add_argument("--cpu-rounds", type=int, default=101, help="CPU baseline rounds (client.cc:368-369: 10 + 101)")
    p.add_argument("--cpu-warmups", type=int, default=10)
    p.add_argument("--cpu-threads", type=int, default=8)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-round", action="store_true",
                   help="N=1: skip the round_world1 object (the N>1 round at world 1, measured after the headline)")
    p.add_argument("--pmc", default="",
                   help="rocprofv3 PMC summary giving HBM traffic per launch (default: the profiles/pmc_*.json "
                        "measured on this workload)")
    p.add_argument("--print-workload", action="store_true", help="print the workload string and exit")
    p.add_argument("--host-resident", action="store_true",
                   help="BASELINE config 5's end-to-end path: the gradient in pinned host memory, reduced in place by "
                        "omr_sparse_buckets_f32 (H2D / scan / exchange / D2H overlapped per bucket); e.g. "
                        "--host-resident --size-mib 4096 --density 0.49")
    p.add_argument("--bucket-mib", type=int, default=256, help="--host-resident: bucket (one round) size")
    p.add_argument("--event-every", type=int, default=10,
                   help="bracket every k-th timed step's kernel with (fence-free) HIP events")
    p.add_argument("--kernel", choices=("fused", "twopass"), default="fused",
                   help="N=1, m=1: single-pass k_scan1f (default) or k_scan1 + k_next")
    p.add_argument("--force-dist", action="store_true",
                   help="take the N>1 (distributed) code path even at WORLD_SIZE=1 (rehearsal under torchrun)")
    p.add_argument("--dist-mode", choices=("reduce", "allreduce", "dense"), default="reduce",
                   help="N>1 step: workers -> aggregators reduce-scatter (BASELINE config 4, default), the full "
                        "all-reduce (sums back to every worker), or the dense stand-in (ncclReduceScatter of the "
                        "whole tensor, C++ driver only)")
    p.add_argument("--dist-pipe", choices=("sync", "async", "defer", "thread", "auto"), default="auto",
                   help="N>1, C++ driver: sync = each round's exchange on the caller's stream; async "
                        "(OMR_ROUND_ASYNC) = round k's exchange over xGMI overlaps round k+1's worker scan; defer "
                        "(OMR_ROUND_DEFER) = as async, and round k's exchange is issued after round k+1's "
                        "first half is queued, so the host never waits for block counts with the GPU idle; thread "
                        "(OMR_ROUND_THREAD | OMR_ROUND_DEFER) = as defer, with everything after the worker scan "
                        "issued by the plan's progress thread; auto (default) = defer or thread, whichever ran the "
                        "untimed probe rounds faster (max over ranks; a round whose host issue time reaches its GPU "
                        "time gains from the thread)")
    p.add_argument("--round-counts", action="store_true",
                   help="N>1 path: ask every round for its block counts (the C API's optional outputs; the step "
                        "reads none)")
    p.add_argument("--pipe-probe", type=int, default=12, help="--dist-pipe auto: untimed rounds per probe trial")
    p.add_argument("--world1-general", action="store_true",
                   help="diagnostic, one rank: time the multi-rank round's code path instead of the one-launch round")
    p.add_argument("--probe-cands", default="",
                   help="diagnostic: the probe's candidates in order, e.g. 'thread:1,defer:2' (pipeline:side streams)")
    p.add_argument("--queue-check", choices=("on", "off"), default="on",
                   help="N>1: check the side streams' hardware queues against the caller's stream (omr_ar_plan_"
                        "set_queue_check; on: the library's default)")
    p.add_argument("--side-streams", choices=("1", "2", "auto"), default="auto",
                   help="N>1: the round's side streams (omr_ar_plan_set_side_streams): one, two (plan + exchange), or "
                        "auto = measured on the node by the probe, with the pipeline mode")
    p.add_argument("--dist-sync", action="store_true", help="same as --dist-pipe sync")
    p.add_argument("--dist-transport", choices=("rccl", "ipc"), default="rccl",
                   help="N>1 round transport: RCCL over xGMI, one process per GPU (the product path), or HIP IPC "
                        "between processes that may share a GPU (a rehearsal of the N>1 path on one GPU; the "
                        "torch.distributed group is then gloo and only carries the id, barriers and timings)")
    return p.parse_args(argv)


def launch_plan(args, env, device_count: int):
    """How this invocation runs ("how N>1 lines are launched"), decided before any GPU call:
    ("run", n_gpus)     this process is the measurement (N=1, or one rank of a launched job); n_gpus is the number of
                        GPUs whose ranks ran, the figure the line reports;
    ("spawn", argv)     --gpus N > 1 without a launcher: start torch.distributed.run with N ranks as a child;
    ("error", message)  refused: never report an N-GPU figure that N GPUs did not produce.
    `value` is always the bytes all ranks processed over the max-over-ranks time, never N x one GPU's rate."""
    launched = "WORLD_SIZE" in env
    ws = int(env.get("WORLD_SIZE", "1"))
    ipc = args.dist_transport == "ipc"
    if not launched:
        n = 1 if args.gpus is None else args.gpus
        if n < 1:
            return "error", f"--gpus {n}: at least one GPU"
        if n == 1:
            return "run", 1
        if not args.host_resident and args.workers != 1:
            return "error", "--workers > 1 is the single-GPU m-worker sum (N=1 only)"
        if device_count < n:
            return "error", (f"--gpus {n} but this node has {device_count} GPU(s): an N-GPU line needs N GPUs, one "
                             f"rank each (nothing was measured)")
        return "spawn", ["--nnodes=1", "--nproc-per-node", str(n), "--master-addr", "127.0.0.1"]
    if args.gpus is not None and args.gpus != ws:
        return "error", f"--gpus {args.gpus} but the launcher started {ws} rank(s)"
    if ipc:  # ranks share the node's GPUs (a rehearsal): the line counts the GPUs, not the ranks
        return "run", max(1, min(ws, device_count))
    if ws > device_count and device_count > 0:
        return "error", f"{ws} RCCL ranks on {device_count} GPU(s): RCCL runs one rank per GPU"
    return "run", ws


def spawn_ranks(torchrun_args, argv) -> int:
    """Run this bench as `torchrun_args` ranks under torch.distributed.run, a child process started before this one
    has made any GPU call (never exec'd over it); rank 0's JSON line is relayed on stdout, everything else on
    stderr.  Returns the child's exit code."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free rendezvous port on the loopback address
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run"] + torchrun_args + ["--master-port", str(port),
                                                                              os.path.abspath(__file__)] + list(argv)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    print(f"bench.py: launching {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in p.stdout:
        (sys.stdout if line.startswith("{") else sys.stderr).write(line)
        (sys.stdout if line.startswith("{") else sys.stderr).flush()
    return p.wait()


def workload_string(args, m: int) -> str:
    return (f"{args.size_mib} MiB fp32 per rank, block_size={args.block_size}, -r {args.density}, {m} worker(s) "
            f"per GPU, device-resident scan+sum")


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def algorithmic_scan_bytes(L: Layout, bitmaps, m: int) -> int:
    """Bytes k_scan1/k_scanm must move per launch: read m*S, write the summed blocks (union non-zero blocks
    and lane heads), the m int32 flag arrays and the row masks."""
    nb, B = L.nb, L.block_size
    union = np.zeros(nb, dtype=bool)
    for bm in bitmaps:
        union |= bm.astype(bool)
    heads = ((np.arange(nb) // L.num_lanes) % L.rows_per_part) == 0
    written = int(np.count_nonzero(union | heads))
    masks = (m if m == 1 else m + 1) * L.rows * 8
    return m * L.nbytes + written * B * 4 + m * nb * 4 + masks


def fused_bytes(L: Layout, bm) -> int:
    """k_scan1f per launch: read S, write the aggregated blocks (non-zero + lane heads), int32 flags and uint32
    next offsets for every block (S + d*S + nb*8, plus the head blocks)."""
    nb, B = L.nb, L.block_size
    heads = ((np.arange(nb) // L.num_lanes) % L.rows_per_part) == 0
    written = int(np.count_nonzero(bm.astype(bool) | heads))
    return L.nbytes + written * B * 4 + nb * 8


def scan_only_bytes(L: Layout) -> int:
    """The round's worker scan (N>1, omr_worker_scan_f32, no sum): read S, write int32 flags, uint32 next
    offsets and uint64 row masks."""
    return L.nbytes + L.nb * 8 + L.rows * 8


def one_rank_round_bytes(L: Layout, bm) -> int:
    """The one-rank round's single launch (omr_worker_scan_tally_f32): fused_bytes, plus one 8-byte tally slot per
    workgroup written, and the previous round's slots read by workgroup 0 to publish its counts (no row masks)."""
    from omr import _lib
    slots = int(_lib.load().omr_tally_slots(L.n, L.block_size, L.num_lanes, L.num_threads))
    return fused_bytes(L, bm) + 2 * slots * 8


def scan_pack_bytes(L: Layout, bm: np.ndarray, rank: int, world: int) -> int:
    """The round's worker scan with the fused pack (omr_worker_scan_pack_f32): scan_only_bytes plus the rank's
    non-zero blocks of the other shards written to their send streams, and the position-table entries of the
    segments it packs (uint32 per (segment, 64-row group, lane))."""
    bounds = [s * L.rows // world for s in range(world + 1)]
    rowmask = np.ones(L.rows, dtype=bool)
    rowmask[bounds[rank]:bounds[rank + 1]] = False
    packed = int(np.count_nonzero(bm.reshape(L.rows, L.num_lanes)[rowmask]))
    from omr import _lib
    import ctypes
    S, gps, ent = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint64()
    _lib.load().omr_pack_geometry(L.n, L.block_size, L.num_lanes, L.num_threads, ctypes.byref(S), ctypes.byref(gps),
                                  ctypes.byref(ent))
    table = ent.value * 4 * (world - 1) // world
    return scan_only_bytes(L) + packed * L.block_size * 4 + table


def step_algorithmic_bytes(L: Layout, bitmaps, m: int) -> int:
    """m*S + d_union*S + m*nb*8 (flag + next per block per worker)."""
    nb = L.nb
    union = np.zeros(nb, dtype=bool)
    for bm in bitmaps:
        union |= bm.astype(bool)
    return m * L.nbytes + int(np.count_nonzero(union)) * L.block_size * 4 + m * nb * 8


def read_pmc(path: str, workload: str, dist_mode: bool):
    """(HBM bytes per launch, source file) from a tools/pmc_traffic.py summary measured on this workload in this
    mode: `path` if given, else the first of profiles/pmc_*.json that matches (the round's worker scan writes no
    aggregated blocks, so single-GPU traffic does not describe it)."""
    cands = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")), reverse=True)
    for c in cands:
        try:
            with open(c) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        same_mode = ("--force-dist" in d.get("bench_args", [])) == dist_mode
        if d.get("workload") == workload and same_mode:
            return d.get("hbm_bytes_per_launch"), c
    return None, None


def read_pmc_round(world: int, L: Layout):
    """(HBM bytes per launch, source) of the N>1 round's worker scan with the fused pack, from tools/pmc_round.py's
    newest summary (profiles/pmc_round_r*.json): measured at config 4's shapes as rank 0 of 8, so it describes only a
    world-8 line over 256 MiB, B=256."""
    if world != 8 or L.nbytes != 256 << 20 or L.block_size != 256:
        return None, None
    paths = (glob.glob(os.path.join(ROOT, "profiles", "pmc_round_r*.json")) +
             glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_round_r*.json")))
    for path in sorted(paths, key=os.path.basename, reverse=True):  # newest round (profiles/rNN/ since round 5)
        try:
            with open(path) as f:
                k = json.load(f)["kernels"]
            kk = next((n for n in ("scan + fused pack + round-check slots (the round's, round 6)",
                                   "scan + fused pack (product)") if n in k), None)  # (the round's own form first)
            return k[kk]["hbm_bytes_per_launch"], path
        except (OSError, ValueError, KeyError):
            continue
    return None, None


def cpu_baseline(L: Layout, bm: np.ndarray, args):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only (never the product path)
    x = oracle.fill(bm, L.block_size)
    t, _, _, _ = oracle.cpu_baseline(x, bm, L.n, L.block_size, L.num_lanes, L.num_threads, args.cpu_threads, 1,
                                     args.cpu_warmups, args.cpu_rounds)
    cores = oracle.cpu_baseline_cores()
    t_ref, _, _, _ = oracle.cpu_baseline(x, bm, L.n, L.block_size, L.num_lanes, L.num_threads, args.cpu_threads,
                                         0, args.cpu_warmups, args.cpu_rounds)
    t1, _, _, _ = oracle.cpu_baseline(x, bm, L.n, L.block_size, L.num_lanes, L.num_threads, 1, 1, 1, 5)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(L.nbytes / t / 1e9, 3),
        "unit": "GB/s",
        "alg_bw_GiBps_reference_style": round(L.nbytes / t / 2 ** 30, 3),
        "cores": args.cpu_threads,
        "pinned_cores": cores,
        "kind": "port",
        "sample": (f"the workload's tensor ({L.nbytes >> 20} MiB, B={L.block_size}, -r {args.density}), data-derived "
                   f"fp32 scan + next offsets + block aggregate, {args.cpu_warmups} warm-up + {args.cpu_rounds} "
                   f"rounds, {args.cpu_threads} pthreads one per partition (client.cc:384-392)"),
        "ms_per_round": round(t * 1e3, 3),
        "reference_faithful_bitmap_walk": {"value": round(L.nbytes / t_ref / 1e9, 3), "unit": "GB/s",
                                           "ms_per_round": round(t_ref * 1e3, 3),
                                           "note": "reads the generator bitmap, never the zero blocks"},
        "one_thread": {"value": round(L.nbytes / t1 / 1e9, 3), "unit": "GB/s", "ms_per_round": round(t1 * 1e3, 3)},
        "host": {"nproc": os.cpu_count(), "cpu_model": cpu_model},
    }


def end_of_timed_region(device_barrier: bool, barrier: bool):
    """The timed region's closing barrier and synchronize.  Over NCCL (RCCL) the barrier is queued behind every step
    (its collective's stream waits for this rank's current stream, which the round's join() has made wait for the
    side streams) and then waited for: 29 us on MI355X, against 70 us for a synchronize first (a host round trip more;
    profiles/r05/timing/barrier/).  Over gloo (IPC ranks) the barrier is host-only, so the device is synchronised
    first."""
    if device_barrier:
        torch.distributed.barrier()
    else:
        torch.cuda.synchronize()
        if barrier:
            torch.distributed.barrier()
    torch.cuda.synchronize()


def round_world1(args, L: Layout, sets, dev, stream, bm=None, torch_group=True):
    """The N>1 step's own code path at N=1, measured after the headline's timed region (which it does not touch): the
    C++ round (worker scan, mask all-gather, plan, exchange with no peers, the one-rank round's sums written by its
    worker scan, deferred pipeline as bench picks) over a one-rank RCCL communicator.  Its per-round time is the
    like-for-like N=1 point of the 1 -> 8 curve, whose N>=2 lines time the same round.
    torch_group (default): exactly the N>1 lines' measurement -- this bench run as one rank under
    torch.distributed.run (--force-dist), in a child process; its line's figures are returned.  Made in-process
    instead (torch_group False: a one-rank communicator with no torch group, after the headline) the same round ran
    118-154 us instead of 59 on MI355X (profiles/r03/round/queues/), so the process set-up of the N>1 lines is kept."""
    if torch_group:
        return round_world1_child(args)
    from omr import cdist
    # RCCL prints a version banner on stdout when the communicator is made: keep stdout for the one JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        eng = cdist.CppSparseAllreduce(L, dev, transport="rccl1")
    except Exception as e:  # noqa: BLE001  (reported, the headline line still prints)
        return {"error": str(e)[:300]}
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    outs = []
    for xs, out in sets:
        out.copy_(xs[0])  # out-of-place: the shard sums land in `out`, x stays the input
        outs.append(out)
    every = max(1, args.event_every)

    def step(i, timed=False):
        eng.run(sets[i % len(sets)][0][0], out=outs[i % len(sets)], mode=1, async_=True, defer=True,
                time_exchange=timed and i % every == 0)

    for i in range(args.warmup):
        step(i)
    eng.join(stream)
    torch.cuda.synchronize()
    eng.stage_timings()  # (discard the warm-up records)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i, timed=True)
    eng.join(stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    stages, _, _, n_timed = eng.stage_timings()
    eng.close()
    scan_ms = stages["scan"]
    # a one-rank round's worker scan writes the shard sums itself (0.0f + x over the write set: omr_sparse_round_f32)
    sb = one_rank_round_bytes(L, bm) if bm is not None else scan_only_bytes(L)
    return {"ms_per_round": round(dt * 1e3, 5), "value": round(L.nbytes / dt / 1e9, 2), "unit": "GB/s",
            "mode": "reduce-scatter (the N>1 bench default), deferred pipeline (OMR_ROUND_DEFER)",
            "transport": "RCCL, one-rank communicator made in this process, no torch group (no peers)",
            "scan_in_round": {"kernel_ms": round(scan_ms, 5), "algorithmic_bytes_per_launch": sb,
                              "frac": round(sb / (scan_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if scan_ms > 0 else None},
            "stages_ms": {k: round(v, 5) for k, v in stages.items()}, "timed_rounds": n_timed}


def round_world1_child(args):
    """bench.py --force-dist as one rank under torch.distributed.run, in a child process (started as a child, never
    exec'd over this GPU process): the N>1 lines' own measurement at world 1.  Returns its figures."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           "--nproc-per-node", "1", os.path.join(ROOT, "bench.py"), "--force-dist", "--no-cpu",
           "--steps", str(max(args.steps, 50)), "--warmup", str(max(args.warmup, 10)),
           "--size-mib", str(args.size_mib), "--block-size", str(args.block_size), "--density", str(args.density)]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    except subprocess.TimeoutExpired:
        return {"error": "the world-1 round's child run timed out (240 s)"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        err = r.stderr or r.stdout
        k = err.find("Traceback")
        return {"error": f"child exit {r.returncode}: " + (err[k:k + 2000] if k >= 0 else err[-600:])}
    d = json.loads(lines[-1])
    ex = d.get("exchange", {})
    rf = d.get("roofline", {})
    return {"ms_per_round": d["ms_per_step"], "value": d["value"], "unit": d["unit"],
            "rounds": d["steps"], "warmup": d["warmup"],
            "mode": "reduce-scatter (the N>1 bench default), pipeline " + str(ex.get("pipe")),
            "transport": "RCCL, one rank under torch.distributed.run (bench.py --force-dist; no peers)",
            "scan_in_round": {"kernel_ms": rf.get("kernel_ms"), "algorithmic_bytes_per_launch":
                              rf.get("algorithmic_bytes_per_launch"), "frac": rf.get("frac"),
                              "traffic": rf.get("traffic"), "traffic_source": rf.get("traffic_source")},
            "stages_ms": ex.get("stages_ms"), "host_ms_per_call": ex.get("host_ms_per_call"),
            "host_wait_ms_per_call": ex.get("host_wait_ms_per_call"),
            "host_issue_ms_per_call": ex.get("host_issue_ms_per_call"),
            "note": ("the N=1 anchor of the per-GPU scaling fraction: the N>=2 lines' measurement at world 1 (a child "
                     "process, run after the headline's timed region)")}


def host_resident(args, ws, rank, local):
    """Config 5: a size-mib gradient per rank in pinned host memory, all-reduced in place bucket by bucket; one step
    = one omr_sparse_buckets_f32 call, which returns when the host buffer holds the result (PCIe both ways
    included).  N=1: a one-rank group (no peers); N>1: RCCL over xGMI between the ranks' staged buckets."""
    from omr import cdist
    dist_mode = ws > 1
    ipc = dist_mode and args.dist_transport == "ipc"  # a rehearsal: ranks share the box's GPUs over HIP IPC
    if dist_mode:
        local = local % max(1, torch.cuda.device_count()) if ipc else local
        torch.cuda.set_device(local)
        if ipc:
            torch.distributed.init_process_group("gloo")
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if dist_mode else 0)
    Lb = Layout.from_bytes(args.bucket_mib << 20, args.block_size)
    total = Layout.from_bytes(args.size_mib << 20, args.block_size)
    bm = ops.gen_bitmap(rank, args.density, total.nb)
    host = ops.fill_blocks(torch.from_numpy(bm).to(dev), total).cpu().pin_memory()
    if ipc:
        uid = [cdist.ipc_unique_id() if rank == 0 else None]
        torch.distributed.broadcast_object_list(uid, src=0)
        eng = cdist.CppSparseAllreduce(Lb, dev, transport="ipc", uid=uid[0], rank=rank, world=ws)
    else:
        eng = cdist.CppSparseAllreduce(Lb, dev, transport="rccl" if dist_mode else "local1")
    step = lambda: eng.run_buckets(host, mode=cdist.CppSparseAllreduce.ALLREDUCE)  # noqa: E731
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist_mode:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    end_of_timed_region(dist_mode and not ipc, dist_mode)
    elapsed = time.perf_counter() - t0
    if dist_mode:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if ipc else dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    # the link's own ceiling on this box: one plain pinned H2D and one D2H of a bucket
    dbuf = torch.empty(Lb.n, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(); dbuf.copy_(host[:Lb.n], non_blocking=True); ev[1].record()
    ev[2].record(); host[:Lb.n].copy_(dbuf, non_blocking=True); ev[3].record()
    torch.cuda.synchronize()
    h2d = Lb.nbytes / (ev[0].elapsed_time(ev[1]) * 1e-3) / 1e9
    d2h = Lb.nbytes / (ev[2].elapsed_time(ev[3]) * 1e-3) / 1e9
    eng.close()
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        # RCCL: one rank per GPU (launch_plan); IPC: the ranks share the box's GPUs
        n_gpus = max(1, min(ws, torch.cuda.device_count())) if ipc else max(ws, 1)
        # (omr_sparse_buckets_f32 reads and writes the mapped pinned buckets in place unless a staging mode is set)
        direct = (not dist_mode and not os.environ.get("OMR_BUCKETS_STAGED")
                  or dist_mode and bool(os.environ.get("OMR_BUCKETS_DIRECT"))) and not any(
            os.environ.get(k) for k in ("OMR_BUCKETS_STAGED_D2H", "OMR_BUCKETS_SCAN_HOST"))
        value = max(ws, 1) * total.nbytes / (ms * 1e-3) / 1e9
        nz = float(bm.mean())
        print(json.dumps({
            "metric": (f"GB/s end-to-end sparse all-reduce from pinned host memory, {args.size_mib} MiB fp32 @ "
                       f"{round(100 * (1 - nz))}% block-sparse per rank (H2D + D2H included)"),
            "value": round(value, 2), "unit": "GB/s", "n_gpus": n_gpus, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (reference generator client.cc:396-421: srand(rank+1), -r {args.density}, 0.01f)",
            "config": {"workload": (f"{args.size_mib} MiB fp32 per rank in pinned host memory, block_size="
                                    f"{args.block_size}, -r {args.density}, buckets of {args.bucket_mib} MiB, "
                                    f"all-reduce in place (BASELINE config 5)"),
                       "parallelism": (f"dp{ws} over HIP IPC, {ws} ranks on {n_gpus} GPU(s): a rehearsal, not a "
                                       f"scaling figure" if ipc else f"dp{n_gpus}"),
                       "ranks": max(ws, 1), "nonzero_fraction": round(nz, 5)},
            "roofline": None,
            "pcie": {"per_rank_GBps": round(total.nbytes / (ms * 1e-3) / 1e9, 2),
                     "plain_h2d_GBps": round(h2d, 2), "plain_d2h_GBps": round(d2h, 2),
                     "spec_GBps": 63.0,
                     "write_back": ("staged: the whole bucket copied back" if os.environ.get("OMR_BUCKETS_STAGED_D2H")
                                    else "zero-copy: the rounds store the write set (union + lane heads) into the "
                                         "pinned buffer"),
                     "read_in": ("direct: each bucket's round reads it from the mapped pinned buffer (the worker "
                                 "scan over PCIe; N > 1: its pack writes the other shards' blocks to device send "
                                 "buffers), no staging copy" if direct else
                                 "staged: H2D copy of each bucket beside the previous bucket's round"),
                     "note": "per rank, over its own PCIe Gen5 x16 link: S in, the write set out"},
            "cpu_baseline": None}), flush=True)
    if dist_mode:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    if args.print_workload:
        print(workload_string(args, args.workers if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 1))
        return
    # (torch.cuda.device_count() does not initialise the GPU on this image: a child may still be started after it)
    how, what = launch_plan(args, os.environ, torch.cuda.device_count())
    if how == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if how == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))
    n_gpus = what
    ws, rank, local = dist_env()
    ranks = ws  # ranks that run the step (each processes its own tensor); n_gpus = the GPUs they ran on
    if args.host_resident:
        host_resident(args, ws, rank, local)
        return
    dist_mode = ws > 1 or args.force_dist
    ipc = dist_mode and args.dist_transport == "ipc"
    if ipc:  # ranks may share GPUs: rank r on GPU r mod count; gloo for the id broadcast, barriers and timings
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("gloo")
    elif dist_mode:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if dist_mode else 0)
    tdev = torch.device("cpu") if ipc else dev  # where the torch.distributed timing reduction runs
    L = Layout.from_bytes(args.size_mib << 20, args.block_size)
    m = args.workers if not dist_mode else 1
    workload = workload_string(args, m)

    # ---- inputs (reference generator, seed = worker id + 1: client.cc:396) -------------------------------
    worker_ids = [rank * m + w for w in range(m)]
    bitmaps = [ops.gen_bitmap(wid, args.density, L.nb) for wid in worker_ids]
    sets = []
    for _ in range(max(1, args.rotate)):
        xs = [ops.fill_blocks(torch.from_numpy(bm).to(dev), L, mode=0) for bm in bitmaps]
        sets.append((xs, torch.zeros(L.n, dtype=torch.float32, device=dev)))
    torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    if dist_mode:
        from omr import cdist
        if ipc:
            uid = [cdist.ipc_unique_id() if rank == 0 else None]
            torch.distributed.broadcast_object_list(uid, src=0)
            engine = cdist.CppSparseAllreduce(L, dev, transport="ipc", uid=uid[0], rank=rank, world=ws)
        else:
            engine = cdist.CppSparseAllreduce(L, device=dev)
        if args.world1_general and ws == 1:
            # diagnostic: the multi-rank round's code path at world 1 (all-gather, plan, exchange as RCCL calls, on the
            # N>1 side streams) instead of the one-launch round
            engine.test_world1_round(True)
            engine.replan()
        if args.queue_check == "off":
            engine.set_queue_check(False)
        engine_fused = engine.fused_pack  # the worker scan packs the exchange's blocks itself
        for xs, out in sets:  # out-of-place result buffers keep every step's input pristine
            out.copy_(xs[0])

        pipe = "sync" if args.dist_sync else args.dist_pipe
        pipe_probe = None  # --dist-pipe auto: the probe's per-round times (ms, max over ranks) per candidate

        host_s = [0.0, 0]  # host time inside engine.run over the timed steps, and their count

        def step(i, ev=None, timed_region=False):
            xs, out = sets[i % len(sets)]
            # a timed step (ev given) brackets each stage of its round (worker scan, bookkeeping, exchange,
            # aggregation) with HIP events on the streams they run on, inside the timed region
            # (omr_ar_plan_stage_timings)
            h0 = time.perf_counter()
            # (the step reads no block counts: a one-rank round then never waits on the host for them)
            engine.run(xs[0], out=out, mode={"allreduce": 0, "reduce": 1, "dense": 2}[args.dist_mode],
                       async_=pipe != "sync", defer=pipe in ("defer", "thread"), thread=pipe == "thread",
                       time_exchange=ev is not None, counts=args.round_counts)
            if timed_region:
                host_s[0] += time.perf_counter() - h0
                host_s[1] += 1
    else:
        fused = m == 1 and args.kernel == "fused"
        plan = ops.ScanSumPlan(L, m, device=dev, fused=fused)
        # the fused step's launch with its arguments converted once per buffer set: one C call per step, in place
        # as the reference returns results into res->buf (client.cc:89)
        launches = [plan.bind(xs[0], xs[0], stream) for xs, _ in sets] if fused else None

        def step(i, ev=None, timed_region=False):
            xs, out = sets[i % len(sets)]
            if m == 1:
                out = xs[0]  # in place, as the reference returns results into res->buf (client.cc:89)
            if ev is not None:
                ev[0].record(stream)
            if launches is not None:
                launches[i % len(sets)]()
            else:
                plan.run(xs, out, with_next=fused)
            if ev is not None:
                ev[1].record(stream)
            if not fused:
                plan.resolve_next()

    def join():  # asynchronous rounds: the caller's stream waits for the last one (the device sync below covers it too)
        if dist_mode:
            engine.join(stream)

    for i in range(args.warmup):
        step(i)
    join()
    torch.cuda.synchronize()
    if dist_mode:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    if dist_mode and pipe == "auto" and args.pipe_probe < 1:
        pipe = "defer"
    side = None  # the side streams the timed rounds ran on (N>1: measured on the node)
    # (auto: both, timed on the node; IPC ranks share GPUs, where a second side stream's hardware queue per rank adds
    # up, so they keep the plan's default of one unless asked)
    sides = (([2, 1] if not ipc else []) if args.side_streams == "auto" else [int(args.side_streams)]
             ) if dist_mode and (ranks > 1 or args.world1_general) else []
    if len(sides) > 1 and args.pipe_probe < 1:  # (no probe rounds: the library's default layout)
        sides = [2]
    if dist_mode and ranks > 1 and pipe != "auto" and len(sides) == 1:
        engine.set_side_streams(sides[0])
        side = sides[0]
    if dist_mode and (pipe == "auto" or len(sides) > 1):
        # untimed probe: the same rounds under each candidate (pipeline mode defer / thread, and at N>1 one or two side
        # streams), alternated twice; every rank takes the candidate with the smaller max-over-ranks round time (so
        # all ranks run one mode)
        pipes = ("defer", "thread") if pipe == "auto" else (pipe,)
        cands = [(pp, sd) for sd in (sides or [None]) for pp in pipes]
        if args.probe_cands:
            cands = [(c.split(":")[0], int(c.split(":")[1]) if sides else None) for c in args.probe_cands.split(",")]
        best = {c: float("inf") for c in cands}
        k = args.warmup
        for _ in range(2):
            for cand in cands:
                pipe = cand[0]
                if cand[1] is not None:
                    engine.set_side_streams(cand[1])
                torch.distributed.barrier()
                t0 = time.perf_counter()
                for _ in range(args.pipe_probe):
                    step(k)
                    k += 1
                join()
                torch.cuda.synchronize()
                dt = torch.tensor([(time.perf_counter() - t0) / args.pipe_probe], dtype=torch.float64, device=tdev)
                torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
                best[cand] = min(best[cand], float(dt.item()))
        # the fastest, except that a candidate earlier in `cands` (defer before thread, two side streams before one)
        # stays chosen unless a later one is more than 3 % faster: the 12-round probe cannot tell a tie apart, and as 4
        # IPC ranks on one GPU a thread-mode tie (1.425 vs 1.426 ms) ran 4.9 ms per round in the timed region
        # (profiles/r05/side_streams/)
        choice = cands[0]
        for c in cands[1:]:
            if best[c] < best[choice] * 0.97:
                choice = c
        pipe, side = choice
        if side is not None:
            engine.set_side_streams(side)
        pipe_probe = {(c[0] if c[1] is None else f"{c[0]}, {c[1]} side stream{'s' if c[1] > 1 else ''}"):
                      round(v * 1e3, 5) for c, v in best.items()}
        torch.distributed.barrier()
        torch.cuda.synchronize()

    from omr import timing
    kev = [(timing.Event(), timing.Event()) for _ in range(args.steps)]
    every = max(1, args.event_every)
    one_kernel = (not dist_mode) and m == 1 and args.kernel == "fused"
    # a one-rank round is ONE launch on the caller's stream (omr_worker_scan_tally_f32): timed as the headline is,
    # events around all K rounds, instead of per-round stage events (a timing record between two rounds holds the next
    # round's launch back 4.6-6 us, profiles/r05/final/w1_trace/; at one rank every other stage is empty)
    one_launch = dist_mode and ranks == 1 and args.dist_mode != "dense" and not args.world1_general
    span = (timing.Event(), timing.Event())  # single-kernel step: the kernel's mean duration over the timed region
    if dist_mode:
        engine.host_stats(reset=True)
    t0 = time.perf_counter()
    if one_kernel or one_launch:
        span[0].record(stream)
    for i in range(args.steps):
        step(args.warmup + i, None if (one_kernel or one_launch) else (kev[i] if i % every == 0 else None),
             timed_region=True)
    if one_kernel or one_launch:
        span[1].record(stream)
    host_wait_us = engine.host_stats(reset=True)[0] if dist_mode else 0.0  # (the timed calls' blocked time only)
    join()
    end_of_timed_region(dist_mode and not ipc, dist_mode)
    elapsed = time.perf_counter() - t0
    if dist_mode:
        t = torch.tensor([elapsed], dtype=torch.float64, device=tdev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3

    roofline = None
    exchange = None
    kernel_name = ("k_scan1f (single pass: scan + sum + next)" if (m == 1 and args.kernel == "fused") else
                   ("k_scan1" if m == 1 else "k_scanm"))
    if dist_mode:
        kernel_name = ("k_scan1f (round worker scan: flags + next + row masks + the fused pack of the other shards' "
                       "blocks)" if engine_fused else
                       "k_scan1f (the one-rank round's single launch: flags + next + the shard sums + per-workgroup "
                       "counts)"
                       if ranks == 1 and args.dist_mode != "dense" else
                       "k_scan1f (round worker scan: flags + next + row masks, no out)")
    scan_ms_dist = None
    if dist_mode:
        # the timed rounds' own events (every `every`-th timed step): its worker scan kernel on the caller's stream,
        # its worker -> aggregator exchange on the stream it ran on
        stages, b_out, b_in, n_timed = engine.stage_timings()
        scan_ms_dist, x_ms = stages["scan"], stages["exchange"]
        exchange = {"ms_mean": round(x_ms, 5), "bytes_out_per_rank": int(b_out), "bytes_in_per_rank": int(b_in),
                    "peers": ws - 1, "timed_rounds": n_timed,
                    "GBps_out_per_rank": round(b_out / (x_ms * 1e-3) / 1e9, 2) if x_ms > 0 else None,
                    "GBps_in_per_rank": round(b_in / (x_ms * 1e-3) / 1e9, 2) if x_ms > 0 else None,
                    "GBps_out_per_peer": (round(b_out / (ws - 1) / (x_ms * 1e-3) / 1e9, 2)
                                          if x_ms > 0 and ws > 1 else None),
                    "xgmi_link_GBps_nominal": XGMI_LINK_GBPS,
                    "timing": (f"HIP events around the worker -> aggregator exchange ({'grouped ncclSend/ncclRecv, dense: ncclReduceScatter' if not ipc else 'the IPC transport copies'}) on the "
                               f"stream it runs on, in every {every}th timed round (inside the timed region), rank 0"),
                    # where a round's time goes (rank 0): each stage's mean from events on its own stream, and the
                    # host time of one engine.run call (a round is host-bound when that exceeds ms_per_step)
                    "stages_ms": {k: round(v, 5) for k, v in stages.items()},
                    "host_ms_per_call": round(host_s[0] / max(1, host_s[1]) * 1e3, 5),
                    # of which blocked on the GPU (the count wait, set reuse, the progress thread): the rest is the
                    # host's own issue time, the figure that says whether a round is host-bound
                    "host_wait_ms_per_call": round(host_wait_us / max(1, host_s[1]) * 1e-3, 5),
                    "host_issue_ms_per_call": round((host_s[0] * 1e6 - host_wait_us) / max(1, host_s[1]) * 1e-3, 5)}
    if not dist_mode:
        kev = kev[::every]
    if one_kernel or one_launch:  # every step is exactly one k_scan1f launch: events around all K steps, divided by K
        kms = span[0].elapsed_time(span[1]) / args.steps
    elif scan_ms_dist is not None:
        kms = scan_ms_dist
    else:
        kms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    if one_launch and exchange is not None:  # (no stage events in a one-rank run: its one stage is the launch)
        exchange["stages_ms"]["scan"] = round(kms, 5)
        exchange["timing"] = ("a one-rank round is one launch on the caller's stream: no per-round stage events; the "
                              "scan stage is the roofline's kernel_ms (events around all K rounds)")
    if dist_mode:
        if ranks == 1 and args.dist_mode != "dense" and args.world1_general:  # (the scan also writes masks)
            kbytes = fused_bytes(L, bitmaps[0]) + L.rows * 8
        elif ranks == 1 and args.dist_mode != "dense":  # one rank: the scan writes the shard sums itself
            kbytes = one_rank_round_bytes(L, bitmaps[0])
        else:
            kbytes = (scan_pack_bytes(L, bitmaps[0], rank, ranks) if engine_fused else scan_only_bytes(L))
    elif m == 1 and args.kernel == "fused":
        kbytes = fused_bytes(L, bitmaps[0])
    else:
        kbytes = algorithmic_scan_bytes(L, bitmaps, m)
    achieved = kbytes / (kms * 1e-3) / 1e9
    if dist_mode and ranks > 1 and engine_fused and args.dist_mode != "dense":
        traffic, pmc_src = read_pmc_round(ranks, L)
    else:
        traffic, pmc_src = read_pmc(args.pmc, workload, dist_mode)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "kernel": kernel_name,
                "kernel_ms": round(kms, 5),
                "algorithmic_bytes_per_launch": kbytes,
                "timing": ("fence-free HIP events (hipEventDisableSystemFence) on the kernel's stream around "
                           "the timed launches" + (" (all K, divided by K)" if one_kernel else
                                                   f" (every {every}th step)")
                           if scan_ms_dist is None else
                           ("fence-free HIP events on the caller's stream around all K timed rounds, divided by K "
                            "(a one-rank round is one launch)") if one_launch else
                           (f"HIP events on the round's stream around its worker scan, in every {every}th timed "
                            f"round (inside the timed region, omr_ar_plan_timings)")),
                "traffic_source": ("rocprofv3 PMC 2*FETCH_SIZE+WRITE_SIZE per launch, "
                                   + os.path.relpath(pmc_src, ROOT)) if traffic else None}
    if not dist_mode:
        sbytes = step_algorithmic_bytes(L, bitmaps, m)
        roofline["step_algorithmic_bytes"] = sbytes
        roofline["step_frac"] = round(sbytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)

    if dist_mode:
        engine_side_streams = engine.side_streams
        engine_queues = engine.queue_report()
        engine.close()  # every rank (the IPC transport's board is released when the last rank leaves)
    if rank != 0:
        if dist_mode:
            torch.distributed.destroy_process_group()
        return
    pipe_note = ""
    if dist_mode and pipe != "sync":
        pipe_note = (", rounds pipelined: exchange k beside scan k+1" +
                     (", exchange k issued after round k+1's first half (OMR_ROUND_DEFER)"
                      if pipe in ("defer", "thread") else "") +
                     (", steps after the scan issued by a progress thread (OMR_ROUND_THREAD)" if pipe == "thread"
                      else ""))
    transport_note = ("RCCL" if not ipc else
                      f"HIP IPC, {ws} ranks on {torch.cuda.device_count()} GPU(s): a rehearsal of the N>1 path, not a "
                      f"scaling figure")
    total_bytes = ranks * m * L.nbytes  # what every rank processed, over the max-over-ranks time
    value = total_bytes / (ms_per_step * 1e-3) / 1e9
    metric = "GB/s device-resident block scan+sum, 256 MiB fp32 @ 90% block-sparse"   # BASELINE.json
    nz = float(np.mean([bm.mean() for bm in bitmaps]))
    if (args.size_mib, args.block_size, args.density) != (256, 256, 0.095):
        # a non-headline config (parity/extra line): name what was actually measured
        metric = (f"GB/s device-resident block scan+sum, {args.size_mib} MiB fp32 @ "
                  f"{round(100 * (1 - nz))}% block-sparse, B={args.block_size}")
    line = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": n_gpus,
        "ranks": ranks,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (reference generator client.cc:396-421: srand(rank+1), -r {args.density}, 0.01f blocks)",
        "config": {"workload": workload, "tensor_bytes_per_rank": L.nbytes, "block_size": L.block_size,
                   "num_lanes": L.num_lanes, "num_threads": L.num_threads, "density_r": args.density,
                   "nonzero_fraction": round(nz, 5),
                   "workers_per_gpu": m, "rotating_buffer_sets": len(sets),
                   "parallelism": "single GPU" if not dist_mode else
                   f"dp{ranks} {dict(allreduce='sparse all-reduce', reduce='sparse reduce-scatter', dense='dense reduce-scatter (stand-in)')[args.dist_mode]} over "
                   f"{transport_note} (C++ round driver, libomr_dist.so{pipe_note})"},
        "alg_bw_GiBps_reference_style": round(total_bytes / (ms_per_step * 1e-3) / 2 ** 30, 2),
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if exchange is not None:
        line["exchange"] = exchange
        line["exchange"]["pipe"] = pipe
        line["exchange"]["side_streams"] = engine_side_streams
        # the side streams' hardware-queue check against the caller's stream (omr_ar_plan_queue_report)
        line["exchange"]["side_stream_queues"] = engine_queues
        if pipe_probe is not None:
            line["exchange"]["pipe_probe_ms_per_round"] = pipe_probe
    if not dist_mode and m == 1 and not args.no_round:
        line["round_world1"] = round_world1(args, L, sets, dev, stream, bitmaps[0])
    if not dist_mode and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(L, bitmaps[0], args)
    print(json.dumps(line), flush=True)
    if dist_mode:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
