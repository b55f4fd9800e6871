#!/usr/bin/env python3
"""Print one round's kernel timeline from a rocprofv3 --kernel-trace CSV (the kernels between two consecutive
launches of the round's first kernel, k_scan1f), plus per-kernel medians over all complete rounds.
usage: python tools/round_timeline.py <..._kernel_trace.csv> [--first k_scan1f] [--round -2]"""
import argparse
import csv
import statistics
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0].replace("void ", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first", default="k_scan1f", help="substring of the round's first kernel")
    ap.add_argument("--round", type=int, default=-2, help="which complete round to print (python index)")
    ap.add_argument("--must", default="k_round_plan", help="only rounds that launch this kernel count")
    a = ap.parse_args()
    with open(a.csv) as f:
        rows = list(csv.DictReader(f))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if a.first in k[2]]
    rounds = [ks[starts[i]:starts[i + 1] + 1] for i in range(len(starts) - 1)]
    rounds = [r for r in rounds if any(a.must in k[2] for k in r)]
    if not rounds:
        sys.exit("no complete round found")
    rd = rounds[a.round]
    t0 = rd[0][0]
    print("# start_us end_us dur_us gap_us name  (last line = next round's first kernel)")
    prev = t0
    for s, e, n in rd:
        print(f"{(s - t0) / 1e3:8.2f} {(e - t0) / 1e3:8.2f} {(e - s) / 1e3:7.2f} {(s - prev) / 1e3:6.2f}  {short(n)}")
        prev = e
    per = [(r[-1][0] - r[0][0]) / 1e3 for r in rounds]
    print(f"# rounds: {len(rounds)}, round period median {statistics.median(per):.2f} us "
          f"(min {min(per):.2f}, max {max(per):.2f})")
    by = {}
    for r in rounds:
        for s, e, n in r[:-1]:
            by.setdefault(short(n), []).append((e - s) / 1e3)
    for n, v in by.items():
        print(f"#   {n:60s} median {statistics.median(v):7.2f} us  x{len(v) / len(rounds):.0f} per round")


if __name__ == "__main__":
    main()
