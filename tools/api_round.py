#!/usr/bin/env python3
"""Host side of a multi-rank round from a rocprofv3 --hip-runtime-trace CSV: per-call median cost of every HIP
API function the bench thread issues between two consecutive k_scan1f launches, and the host time per round.
usage: python tools/api_round.py <..._hip_api_trace.csv> [<..._kernel_trace.csv>]"""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    main_tid = collections.Counter(r["Thread_Id"] for r in rows if r["Function"] == "hipLaunchKernel"
                                   or r["Function"] == "hipExtModuleLaunchKernel").most_common(1)[0][0]
    rows = [r for r in rows if r["Thread_Id"] == main_tid]
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"# thread {main_tid}: {len(rows)} calls over {span / 1e3:.1f} ms")
    for f, v in sorted(by.items(), key=lambda x: -sum(x[1]))[:25]:
        print(f"{f:40s} n={len(v):6d} median={statistics.median(v):8.2f} us  total={sum(v) / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
