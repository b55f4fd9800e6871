#!/usr/bin/env python3
"""Print the bench thread's HIP API calls of one round (between two k_scan1f launches) with their cost and the
host gap before each, joined to the kernels they launched.  usage: api_round_seq.py <dir with tl_*.csv> [round]"""
import csv
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 60
A = list(csv.DictReader(open(f"{d}/tl_hip_api_trace.csv")))
K = {r["Correlation_Id"]: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:28]
     for r in csv.DictReader(open(f"{d}/tl_kernel_trace.csv"))}
A.sort(key=lambda r: int(r["Start_Timestamp"]))
A = [r for r in A if r["Thread_Id"] == r["Process_Id"] and r["Function"] not in
     ("hipThreadExchangeStreamCaptureMode", "hipGetDevice", "hipGetLastError", "hipSetDevice")]
idx = [i for i, r in enumerate(A) if K.get(r["Correlation_Id"], "").startswith("k_scan1f")]
i0, i1 = idx[k], idx[k + 1]
t0 = prev = int(A[i0]["Start_Timestamp"])
for r in A[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.2f} {(e - s) / 1e3:6.2f} gap {(s - prev) / 1e3:6.2f}  {r['Function']:24s} "
          f"{K.get(r['Correlation_Id'], '')}")
    prev = e
