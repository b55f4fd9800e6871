#!/usr/bin/env python3
"""Measure HBM traffic per launch of the dominant kernel with rocprofv3 PMC counters and write the summary
bench.py reads (profiles/pmc_r01.json by default).

Recipe (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and WRITE_SIZE in SEPARATE --pmc
passes (FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2); both are KiB; on gfx950 FETCH_SIZE reports exactly half
of a wide (16 B/lane) coalesced streaming read, so hbm_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16 B/lane streaming stores.  Each pass runs `python bench.py` under rocprofv3 with the counters only
(no --sys-trace / --runtime-trace), from /tmp as the guide asks.

usage: python tools/pmc_traffic.py [--kernel k_scan1] [--also k_round_plan,k_shard_sum_list] [--out ...] [-- bench args]
--also: further kernels of the same run, each reported per launch under "also" (round 6: every kernel of the N>1
path's round at world 1, so the round's HBM bytes can be added up).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir, bench_args):
    cmd = ["rocprofv3", "--pmc", counter, "-d", outdir, "-o", "pmc", "--output-format", "csv", "--",
           sys.executable, os.path.join(ROOT, "bench.py")] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(cmd, check=True, env=env, cwd="/tmp", stdout=subprocess.DEVNULL, timeout=180)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {outdir}")
    return files[0]


def per_launch(csv_path, kernel, counter):
    vals = {}
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"{counter}: no rows for kernel {kernel} in {csv_path}")
    v = sorted(vals.values())
    return sum(v) / len(v), len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_scan1f")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_r01.json"))
    ap.add_argument("--workdir", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    ap.add_argument("--also", default="", help="comma-separated further kernel names, reported per launch")
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    a.out, a.workdir = os.path.abspath(a.out), os.path.abspath(a.workdir)  # the passes run from /tmp
    # (--no-round: bench's N=1 line would otherwise also run its world-1 round in a child process under the profiler)
    bench_args = [x for x in a.bench_args if x != "--"] or ["--steps", "20", "--warmup", "5", "--no-cpu", "--no-round"]
    fetch_csv = run_pass("FETCH_SIZE", os.path.join(a.workdir, "fetch"), bench_args)
    write_csv = run_pass("WRITE_SIZE", os.path.join(a.workdir, "write"), bench_args)
    fetch_kib, nf = per_launch(fetch_csv, a.kernel, "FETCH_SIZE")
    write_kib, nw = per_launch(write_csv, a.kernel, "WRITE_SIZE")
    # the workload string bench.py prints, so bench.py only picks this file up for the same configuration
    probe = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + bench_args + ["--print-workload"],
                           check=True, capture_output=True, text=True).stdout.strip().splitlines()[-1]
    res = {
        "workload": probe,
        "kernel": a.kernel,
        "launches": {"fetch_pass": nf, "write_pass": nw},
        "FETCH_SIZE_kib_per_launch": fetch_kib,
        "WRITE_SIZE_kib_per_launch": write_kib,
        "hbm_read_bytes_per_launch": 2 * fetch_kib * 1024,
        "hbm_write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": int(2 * fetch_kib * 1024 + write_kib * 1024),
        "correction": "read = 2 x FETCH_SIZE (gfx950 16 B/lane streaming reads), write = WRITE_SIZE, KiB",
        "bench_args": bench_args,
    }
    also = {}
    for k in [x for x in a.also.split(",") if x]:
        try:
            fk, nfk = per_launch(fetch_csv, k, "FETCH_SIZE")
            wk, nwk = per_launch(write_csv, k, "WRITE_SIZE")
        except SystemExit:  # (not launched in this run)
            also[k] = None
            continue
        also[k] = {"launches": {"fetch_pass": nfk, "write_pass": nwk}, "hbm_read_bytes_per_launch": 2 * fk * 1024,
                   "hbm_write_bytes_per_launch": wk * 1024, "hbm_bytes_per_launch": int(2 * fk * 1024 + wk * 1024)}
    if also:
        res["also"] = also
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
