"""Per-step kernel breakdown of a rocprofv3 kernel trace, split by step kind (steps are delimited by the sampler
kernel): decode-only steps vs mixed steps (a step that launched any hipBLASLt/rocBLAS GEMM, i.e. T > the streaming
kernel's M limit, or prefill attention items). Usage: ktrace_mix.py trace.csv [nsteps]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
nsteps = min(nsteps, len(idx) - 1)
steps = []
for j in range(len(idx) - nsteps, len(idx)):
    sel = rows[idx[j - 1] + 1: idx[j] + 1]
    steps.append(sel)
kinds = defaultdict(list)
for sel in steps:
    names = [r["Kernel_Name"] for r in sel]
    mixed = any(n.startswith("Cijk") or "Cijk" in n[:10] for n in names)
    kinds["mixed" if mixed else "decode"].append(sel)
tot_wall = 0.0
for kind, ss in sorted(kinds.items()):
    agg = defaultdict(lambda: [0, 0.0])
    wall = 0.0
    for sel in ss:
        wall += (int(sel[-1]["End_Timestamp"]) - int(steps[0][0]["Start_Timestamp"]) * 0 - int(sel[0]["Start_Timestamp"])) / 1e3
        for r in sel:
            name = re.sub(r"\(.*", "", r["Kernel_Name"])[:64]
            agg[name][0] += 1
            agg[name][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n = len(ss)
    tot_wall += wall
    busy = sum(v[1] for v in agg.values())
    print(f"== {kind}: {n} steps, wall {wall / n:.1f} us/step, kernel-busy {busy / n:.1f} us/step, "
          f"{sum(len(s) for s in ss) / n:.0f} kernels/step")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {k:64s} {c / n:6.1f}/step {t / n:9.1f} us/step {100 * t / busy:5.1f}%")
first = int(steps[0][0]["Start_Timestamp"])
last = int(steps[-1][-1]["End_Timestamp"])
print(f"== all: {len(steps)} steps, {(last - first) / 1e3 / len(steps):.1f} us/step end-to-end "
      f"(incl. host gaps between steps)")
