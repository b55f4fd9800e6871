#!/usr/bin/env python3
"""Round 5: summarise the kernel trace of bench.py's N>1 path rehearsed as 8 IPC ranks on one GPU
(tools/gpu_recipes.sh ipc_ranks TAG 8 trace: one rocprofv3 --kernel-trace file per rank): per rank, the GPU time by kernel kind (the round's
kernels, ROCclr's device-side waits for IPC events `__amd_rocclr_streamOpsWait`, its event writes, copies), the hardware
queues each rank used, the fraction of the span its queues and the whole GPU had a kernel running, and rank 0's
per-round intervals (scan to scan).
usage: python tools/ipc_trace_r05.py TRACE_DIR [--json OUT]"""
import argparse
import collections
import csv
import glob
import json
import os


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    return tot + (ce - cs if cs is not None else 0)


def kind(name):
    for k, pat in (("wait (streamOpsWait)", "streamOpsWait"), ("event write (streamOpsWrite)", "streamOpsWrite"),
                   ("copy", "copyBuffer"), ("scan", "k_scan1f"), ("plan", "round_plan"), ("shard sum", "shard_sum")):
        if pat in name:
            return k
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.trace_dir, "rank*_kernel_trace.csv")))
    out = {"ranks": {}}
    allk, allc = [], []
    for f in files:
        r = os.path.basename(f).split("_")[0]
        rows = list(csv.DictReader(open(f)))
        iv = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows]
        s0, e0 = min(s for s, _ in iv), max(e for _, e in iv)
        by = collections.defaultdict(float)
        cnt = collections.Counter()
        for x in rows:
            k = kind(x["Kernel_Name"])
            by[k] += (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
            cnt[k] += 1
        comp = [(int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in rows if "rocclr" not in x["Kernel_Name"]]
        allk += iv
        allc += comp
        scans = sorted(int(x["Start_Timestamp"]) for x in rows if "k_scan1f" in x["Kernel_Name"])
        out["ranks"][r] = {
            "span_ms": round((e0 - s0) / 1e6, 1), "rounds": cnt["scan"],
            "gpu_ms_by_kind": {k: round(v, 1) for k, v in sorted(by.items())},
            "launches_by_kind": dict(cnt),
            "queues": sorted(set(x["Queue_Id"] for x in rows)),
            "queue_busy_frac": round(union(iv) / (e0 - s0), 3),
            "compute_busy_frac": round(union(comp) / (e0 - s0), 3),
            "round_intervals_ms": [round((b - a_) / 1e6, 2) for a_, b in zip(scans, scans[1:])] if r == "rank0" else None,
        }
    s0, e0 = min(s for s, _ in allk), max(e for _, e in allk)
    out["gpu"] = {"span_ms": round((e0 - s0) / 1e6, 1), "any_kernel_frac": round(union(allk) / (e0 - s0), 3),
                  "compute_kernel_frac": round(union(allc) / (e0 - s0), 3)}
    for r, v in out["ranks"].items():
        print(r, {k: v[k] for k in ("span_ms", "rounds", "queues", "queue_busy_frac", "compute_busy_frac")})
        print("   GPU ms:", v["gpu_ms_by_kind"], " launches:", v["launches_by_kind"])
    print("GPU:", out["gpu"])
    print("rank0 round intervals (ms):", out["ranks"]["rank0"]["round_intervals_ms"])
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
