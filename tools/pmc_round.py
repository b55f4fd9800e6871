#!/usr/bin/env python3
"""HBM traffic per launch of the multi-rank round's kernels at config-4 shapes (tools/tune_round_r03.py cases), with
rocprofv3 PMC counters, against their algorithmic bytes.  Recipe as tools/pmc_traffic.py (MI355X_MICROARCH.md
§HBM): FETCH_SIZE and WRITE_SIZE in separate --pmc passes, counters only, from /tmp; read = 2 x FETCH_SIZE KiB
(gfx950, 16 B/lane streaming reads), write = WRITE_SIZE KiB.
usage: python tools/pmc_round.py [--out profiles/r03/pmc_round.json]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [  # (tune_round_r03 case filter, kernel name in the trace)
    ("product k_shard_sum_list", "::k_shard_sum_list<"),
    ("scan + fused pack (product)", "::k_scan1f<"),
    ("scan + fused pack + round-check", "::k_scan1f<"),
    ("round plan as the round calls it (pair", "::k_round_plan<"),
    ("round plan as the round calls it + round check", "::k_round_plan<"),
    ("round plan as the round calls it, round-3/4", "::k_round_plan_r04("),
    ("round plan, no chain (k_round_plan)", "::k_round_plan<"),
    ("round plan, no chain (round-3/4", "::k_round_plan_r04("),
]
# (the read-request sizes behind FETCH_SIZE: one pass of these TCC counters per case, to calibrate the read bytes of
# kernels whose loads are not 16 B per lane, as the plan's 8-byte mask reads, MI355X_MICROARCH.md HBM section)
REQ_COUNTERS = "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum"
TIMED = 10  # the case's own launches (--rounds 2 --reps 5): the last ones of its kernel in the trace


def last_launches(csv_path, kernel, counter, k=TIMED):
    """Mean counter value per dispatch over the last k dispatches of `kernel` (setup and checking launches of the
    same kernel come first)."""
    import csv
    vals = {}
    with open(csv_path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", "") or row.get("Counter_Name") != counter:
                continue
            d = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"{counter}: no rows for kernel {kernel} in {csv_path}")
    v = [vals[d] for d in sorted(vals)][-k:]
    return sum(v) / len(v), len(v)


def run_pass(counter, outdir, case):
    cmd = ["rocprofv3", "--pmc", *counter.split(), "-d", outdir, "-o", "pmc", "--output-format", "csv", "--",
           sys.executable, os.path.join(ROOT, "tools", "tune_round_r03.py"), "--only", case, "--rounds", "2",
           "--reps", "5"]
    subprocess.run(cmd, check=True, env=dict(os.environ, TMPDIR="/tmp"), cwd="/tmp", stdout=subprocess.DEVNULL,
                   timeout=240)
    import glob
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {outdir}")
    return files[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "pmc_round.json"))
    ap.add_argument("--workdir", default=os.path.join(ROOT, "gpurun_out", "pmc_round"))
    ap.add_argument("--only", default="", help="only the cases whose filter contains this")
    a = ap.parse_args()
    a.out, a.workdir = os.path.abspath(a.out), os.path.abspath(a.workdir)
    os.makedirs(a.workdir, exist_ok=True)
    res = {}
    for case, kernel in CASES:
        if a.only and a.only not in case:
            continue
        tag = case.split()[0] + "_" + str(abs(hash(case)) % 1000)
        alg = os.path.join(a.workdir, tag + "_alg.json")
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tune_round_r03.py"), "--only", case, "--rounds",
                        "3", "--reps", "10", "--json", alg], check=True, timeout=240, stdout=subprocess.DEVNULL)
        with open(alg) as f:
            rep = json.load(f)
        name = next(k for k in rep if case in k)
        fcsv = run_pass("FETCH_SIZE", os.path.join(a.workdir, tag, "fetch"), case)
        wcsv = run_pass("WRITE_SIZE", os.path.join(a.workdir, tag, "write"), case)
        fk, nf = last_launches(fcsv, kernel, "FETCH_SIZE")
        wk, nw = last_launches(wcsv, kernel, "WRITE_SIZE")
        qcsv = run_pass(REQ_COUNTERS, os.path.join(a.workdir, tag, "req"), case)
        req = {c: last_launches(qcsv, kernel, c)[0] for c in REQ_COUNTERS.split()}
        n, n128, n32, n64 = (req[c] for c in REQ_COUNTERS.split())
        hbm = 2 * fk * 1024 + wk * 1024
        res[name] = {"kernel": kernel, "launches": {"fetch_pass": nf, "write_pass": nw},
                     "hbm_read_bytes_per_launch": int(2 * fk * 1024), "hbm_write_bytes_per_launch": int(wk * 1024),
                     "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes": rep[name]["algorithmic_bytes"],
                     "pmc_over_algorithmic": round(hbm / rep[name]["algorithmic_bytes"], 4),
                     "read_requests": {"TCC_EA0_RDREQ": n, "TCC_BUBBLE (128 B)": n128, "_32B": n32, "_64B": n64,
                                       "bytes_by_request_size": int(128 * n128 + 64 * n64 + 32 * n32)},
                     "us": rep[name]["us"]}
        print(json.dumps({name: res[name]}), flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"shapes": "config 4: 8 workers x 256 MiB, -r 0.095, shard 0 of 8 (tools/tune_round_r03.py)",
                   "correction": "read = 2 x FETCH_SIZE (gfx950 16 B/lane streaming reads), write = WRITE_SIZE, KiB; "
                                 "read_requests: the TCC_EA0_RDREQ counts (all, 32-byte, 64-byte) behind FETCH_SIZE",
                   "kernels": res}, f, indent=1)


if __name__ == "__main__":
    main()
