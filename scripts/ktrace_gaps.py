"""Inter-kernel gaps of the last `nsteps` pure-decode engine steps of a rocprofv3 kernel trace: for every consecutive
kernel pair (previous kernel -> kernel, short names) the mean gap (start - previous end) per step, plus the total.
Comparing two traces (eager vs hipGraph replay) shows WHICH boundaries grow. Usage: ktrace_gaps.py trace.csv [nsteps]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
nsteps = min(nsteps, len(idx) - 1)
steps = [rows[idx[i] + 1:idx[i + 1] + 1] for i in range(len(idx) - nsteps - 1, len(idx) - 1)]
steps = [st for st in steps if not any("Cijk" in r["Kernel_Name"] or "skinny" in r["Kernel_Name"] for r in st)]


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)
    m = re.match(r"_ZN5kafka\d+(\w+?)I", n)
    if m:
        n = m.group(1)
    n = n.replace("kafka::", "")
    return n[:40]


agg = defaultdict(lambda: [0, 0.0])
total = 0.0
for st in steps:
    for a, b in zip(st, st[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        k = (short(a["Kernel_Name"]), short(b["Kernel_Name"]))
        agg[k][0] += 1
        agg[k][1] += g
        total += g
n = max(1, len(steps))
print(f"decode steps {len(steps)}: gaps {total / n:.1f} us/step over {sum(v[0] for v in agg.values()) / n:.1f} "
      f"boundaries")
for (a, b), (c, s) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"  {a:40s} -> {b:40s} {c / n:6.1f}/step  {s / c:6.2f} us/gap  {s / n:7.1f} us/step")
