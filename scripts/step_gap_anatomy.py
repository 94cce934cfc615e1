#!/usr/bin/env python3
"""Anatomy of each engine step's start gap from one rocprofv3 run with --kernel-trace --hip-trace: for the first
kernel after the step's plan upload (the copyBuffer that follows the previous step's token download), when was it
ENQUEUED (its HIP launch call, matched by correlation id) relative to the moment the GPU went idle? A launch call
that ends after the GPU went idle means the host was late; one that ended before means the kernel sat queued.
Usage: step_gap_anatomy.py <rocprofv3 output dir> [last N steps]"""
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kt = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
    ht = sorted(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True))[0]
    ks = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    api = {}
    for r in csv.DictReader(open(ht)):
        api[r["Correlation_Id"]] = r
    idx = [i for i, r in enumerate(ks) if "sample_kernel" in r["Kernel_Name"]]
    rows = []
    for a, b in zip(idx[-last - 1:-1], idx[-last:]):
        st = ks[a + 1:b + 1]
        # the largest gap of the step and the kernel after it
        best = max(range(1, len(st)), key=lambda j: int(st[j]["Start_Timestamp"]) - int(st[j - 1]["End_Timestamp"]))
        prev, k = st[best - 1], st[best]
        idle_from = int(prev["End_Timestamp"])
        gap = (int(k["Start_Timestamp"]) - idle_from) / 1e3
        call = api.get(k["Correlation_Id"])
        if call is None:
            continue
        enq_end = (int(call["End_Timestamp"]) - idle_from) / 1e3
        enq_start = (int(call["Start_Timestamp"]) - idle_from) / 1e3
        rows.append((gap, enq_start, enq_end, prev["Kernel_Name"][:30], k["Kernel_Name"][:30], call["Function"]))
    for g, s, e, p, k, f in rows:
        print(f"gap {g:7.1f} us  launch call {s:8.1f} .. {e:8.1f} us rel. to idle  after {p} -> {k} ({f})")
    if rows:
        print(f"== median gap {statistics.median(r[0] for r in rows):.1f} us, median launch-call end "
              f"{statistics.median(r[2] for r in rows):.1f} us after the GPU went idle")


if __name__ == "__main__":
    main()
