#!/usr/bin/env python3
"""Per-kernel busy time and inter-kernel gaps per pure decode step of two rocprofv3 kernel traces (e.g. eager vs
hipGraph replay of the headline). Usage: ktrace_compare.py A/run_kernel_trace.csv B/run_kernel_trace.csv [steps]"""
import collections
import csv
import re
import sys


def load(f, nsteps):
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
    steps = [rows[idx[i] + 1:idx[i + 1] + 1] for i in range(max(0, len(idx) - nsteps - 1), len(idx) - 1)]
    agg, cnt, n, gaps, walls = collections.Counter(), collections.Counter(), 0, 0.0, 0.0
    for st in steps:
        if any("Cijk" in r["Kernel_Name"] or "skinny" in r["Kernel_Name"] for r in st):
            continue
        if any("attn_tile" in r["Kernel_Name"] and int(r["Grid_Size_Y"]) != 32 for r in st):
            continue  # a new turn's prefill tiles: not a pure decode step
        n += 1
        for r in st:
            k = re.sub(r"\(.*", "", r["Kernel_Name"])[:50]
            agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
        gaps += sum(max(0, int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) for a, b in zip(st, st[1:])) / 1e3
        walls += (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
    return {k: v / n for k, v in agg.items()}, {k: v / n for k, v in cnt.items()}, gaps / n, walls / n, n


def main():
    ns = int(sys.argv[3]) if len(sys.argv) > 3 else 56
    a, ac, ag, aw, an = load(sys.argv[1], ns)
    b, bc, bg, bw, bn = load(sys.argv[2], ns)
    print(f"pure decode steps {an} / {bn}; wall {aw:.1f} / {bw:.1f} us; gaps {ag:.1f} / {bg:.1f} us per step; "
          f"kernels {sum(ac.values()):.1f} / {sum(bc.values()):.1f}")
    for k in sorted(set(a) | set(b), key=lambda k: -(a.get(k, 0) + b.get(k, 0))):
        print(f"{k:50s} {a.get(k, 0):8.1f} ({ac.get(k, 0):5.1f})  {b.get(k, 0):8.1f} ({bc.get(k, 0):5.1f})  "
              f"diff {b.get(k, 0) - a.get(k, 0):7.1f}")


if __name__ == "__main__":
    main()
