"""Per-step kernel breakdown of the LAST `nsteps` engine steps of a rocprofv3 kernel trace (steps are delimited by
the sampler kernel). Usage: ktrace.py trace.csv [nsteps]"""
import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
if len(idx) <= nsteps:
    nsteps = len(idx) - 1
a, b = idx[-nsteps - 1] + 1, idx[-1] + 1
sel = rows[a:b]
agg = defaultdict(lambda: [0, 0.0])
for r in sel:
    name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[name][0] += 1
    agg[name][1] += d
wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"last {nsteps} steps: wall {wall/nsteps:.1f} us/step, kernel-busy {busy/nsteps:.1f} us/step, {len(sel)/nsteps:.0f} kernels/step")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    grid = ""
    print(f"{k:60s} {c/nsteps:6.1f}/step {t/nsteps:9.1f} us/step {100*t/busy:5.1f}%")
