#!/usr/bin/env python3
"""Per-kernel mean PMC counters + MFMA utilisation from rocprofv3 --pmc CSVs (scripts/gpu_pmc_mfma.sh).

MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs x SIMDs): the busy counter sums matrix-pipe cycles
over all SIMDs (32 per v_mfma_f32_32x32x16_bf16 = SQ_INSTS_MFMA x 32), GRBM_GUI_ACTIVE sums the active cycles of the
8 XCDs (per XCD it matches the kernel's duration x clock). Usage:
pmc_mfma_summary.py <dir with run_counter_collection.csv> [simds=1024] [xcds=8]"""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
simds = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
xcds = int(sys.argv[3]) if len(sys.argv) > 3 else 8
for f in sorted(root.rglob("run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if "kafka" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0][:60]
        acc[(name, r["Dispatch_Id"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (name, _), cs in acc.items():
        for c, v in cs.items():
            per[name][c].append(sum(v))
    print(f"== {f.parent.name}")
    for name, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        util = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1.0, m.get("GRBM_GUI_ACTIVE", 1) / xcds * simds)
        wait = m.get("SQ_WAIT_ANY", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 1))
        print(f"  {name:60s} n={len(next(iter(cs.values())))} MFMA util {100 * util:5.1f} %  "
              f"mfma/dispatch {m.get('SQ_INSTS_MFMA', 0):.3g}  active cycles/XCD {m.get('GRBM_GUI_ACTIVE', 0) / xcds:.3g}  "
              f"wait_any/wave_cycles {100 * wait:4.1f} %")
