#!/usr/bin/env python3
"""Host/GPU timeline of bench steps from one rocprofv3 run with --kernel-trace --marker-trace (KAFKA_ROCTX=1):
per step, the GPU time (first kernel start -> sampler end), the kernel-busy time, the idle gaps between kernels,
and for the largest gap which host span (roctx: schedule / plan_ahead / launch / collect) was open when the GPU
went idle. Usage: step_timeline.py <rocprofv3 output dir> [last N steps]"""
from __future__ import annotations

import csv
import glob
import re
import statistics
import sys


def load(d: str):
    kt = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))
    mk = sorted(glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True))
    ks = []
    for f in kt:
        for r in csv.DictReader(open(f)):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"])[:40]))
    ks.sort()
    spans = []
    for f in mk:
        for r in csv.DictReader(open(f)):
            name = r.get("Operation") or r.get("Function") or ""
            msg = r.get("Message") or r.get("Roctx_Message") or name
            try:
                spans.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), msg))
            except (KeyError, ValueError):
                continue
    spans.sort()
    return ks, spans


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    ks, spans = load(d)
    steps, cur = [], []
    for k in ks:
        cur.append(k)
        if "sample_kernel" in k[2]:
            steps.append(cur)
            cur = []
    steps = steps[-last:]
    walls, busies, gaps_tot = [], [], []
    for st in steps:
        t0, t1 = st[0][0], st[-1][1]
        busy = sum(e - s for s, e, _ in st)
        gaps = sorted(((b[0] - a[1], a, b) for a, b in zip(st, st[1:])), reverse=True)
        walls.append((t1 - t0) / 1e3)
        busies.append(busy / 1e3)
        gaps_tot.append(sum(max(0, g) for g, _, _ in gaps) / 1e3)
        g, a, b = gaps[0]
        open_spans = [m for s, e, m in spans if s <= a[1] <= e]
        print(f"step {walls[-1]:8.0f} us busy {busies[-1]:8.0f} gaps {gaps_tot[-1]:6.0f}  largest {g / 1e3:6.0f} us "
              f"after {a[2][:28]} -> {b[2][:28]}; host spans open: {open_spans[:4]}")
    print(f"== {len(steps)} steps: wall p50 {statistics.median(walls):.0f} us, busy p50 {statistics.median(busies):.0f}, "
          f"gaps mean {statistics.mean(gaps_tot):.0f} us/step")


if __name__ == "__main__":
    main()
