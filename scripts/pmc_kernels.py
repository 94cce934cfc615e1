"""Mean PMC counter values per dispatch for each kernel (rocprofv3 --pmc csv) + mean duration from the kernel trace
of the same run. Usage: pmc_kernels.py <dir with *_counter_collection.csv and *_kernel_trace.csv> [name filter]"""
import csv
import glob
import re
import sys
from collections import defaultdict

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
vals = defaultdict(lambda: defaultdict(list))
for f in cc:
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
        if flt and flt not in name:
            continue
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in kt:
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
        if flt and flt not in name:
            continue
        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, cs in vals.items():
    ds = dur.get(name, [])
    print(f"== {name}  dispatches {max(len(v) for v in cs.values())}  mean dur {sum(ds) / max(len(ds), 1):.1f} us")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}")
