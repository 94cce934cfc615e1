"""Per-(kernel, grid) breakdown of the last `nsteps` engine steps of a rocprofv3 kernel trace, decode steps (no
prefill tile kernel with a q-row grid) and mixed steps separately: mean us per call and per step, so the same kernel
on different shapes (the four projections of a layer) is told apart. Usage: ktrace_shapes.py trace.csv [nsteps]"""
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


def grid(r):
    return tuple(int(r.get(k, 0) or 0) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))


kinds = defaultdict(list)
for st in steps:
    mixed = any("Cijk" in r["Kernel_Name"] or "skinny" in r["Kernel_Name"] for r in st)
    kinds["mixed" if mixed else "decode"].append(st)
for kind, sts in kinds.items():
    agg = defaultdict(lambda: [0, 0.0])
    wall = 0.0
    for st in sts:
        wall += (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3
        for r in st:
            name = re.sub(r"\(.*", "", r["Kernel_Name"])[:52]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = agg[(name, grid(r))]
            a[0] += 1
            a[1] += d
    n = len(sts)
    busy = sum(v[1] for v in agg.values())
    # early-launched kernels overlap their predecessors (models/llama.py EARLY): the union of the kernels' intervals
    # is the time the GPU had any kernel resident; the per-kernel sums then include time spent waiting on a gate
    union = 0.0
    for st in sts:
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in st)
        cur_s, cur_e = iv[0]
        for s0, e0 in iv[1:]:
            if s0 > cur_e:
                union += (cur_e - cur_s) / 1e3
                cur_s, cur_e = s0, e0
            else:
                cur_e = max(cur_e, e0)
        union += (cur_e - cur_s) / 1e3
    print(f"== {kind}: {n} steps, wall {wall / n:.1f} us/step, kernel-busy {busy / n:.1f} us/step "
          f"(sum of kernel durations), any-kernel-resident {union / n:.1f} us/step")
    for (k, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"  {k:52s} grid {str(g):22s} {c / n:6.1f}/step {t / c:8.1f} us/call {t / n:9.1f} us/step")
