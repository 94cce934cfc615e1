"""Where a step's extra rows go: a rocprofv3 kernel trace cut into engine steps (each ends with its sample kernel),
matched from the end with the bench's step log (KAFKA_BENCH_STEPLOG: token rows of the step each call launched),
then per kernel family the mean us per step for every rows bucket and its excess over the pure-decode bucket.
Usage: ktrace_rows.py trace.csv steplog.jsonl"""
import csv
import json
import re
import sys
from collections import defaultdict

trace = list(csv.DictReader(open(sys.argv[1])))
trace.sort(key=lambda r: int(r["Start_Timestamp"]))
log = [json.loads(line) for line in open(sys.argv[2])]
ends = [i for i, r in enumerate(trace) if "sample_kernel" in r["Kernel_Name"]]
steps = [trace[ends[i] + 1:ends[i + 1] + 1] for i in range(len(ends) - 1)]
n = min(len(steps), len(log) - 1)
steps, log = steps[-n:], log[-n:]  # the last step's sample kernel closes the log's last record


def family(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)
    m = re.match(r"_ZN5kafka\d+(\w+?)I", n)
    if m:
        n = m.group(1)
    n = n.replace("kafka::", "")
    if n.startswith("Cijk"):
        return "hipBLASLt " + ("MT" + n.split("_MT")[1][:9] if "_MT" in n else n[:20])
    return n[:44]


def bucket(rows: int) -> str:
    for hi in (64, 96, 128, 160, 192, 256):
        if rows <= hi:
            return f"<={hi}"
    return ">256"


agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
tok = defaultdict(int)
for st, rec in zip(steps, log):
    b = bucket(rec.get("rows") or 0)
    cnt[b] += 1
    tok[b] += rec.get("rows") or 0
    for r in st:
        agg[b][family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
order = sorted(cnt, key=lambda b: int(b[2:]) if b[0] == "<" else 10**6)
base = order[0]
fams = sorted({f for b in order for f in agg[b]}, key=lambda f: -max(agg[b][f] / cnt[b] for b in order))
print("bucket  steps  mean rows  kernel-busy us/step  (excess over " + base + ")")
for b in order:
    busy = sum(agg[b].values()) / cnt[b]
    print(f"{b:6s} {cnt[b]:6d} {tok[b] / cnt[b]:10.1f} {busy:12.1f} {busy - sum(agg[base].values()) / cnt[base]:+10.1f}")
print()
print(f"{'kernel family':44s} " + " ".join(f"{b:>16s}" for b in order))
for f in fams[:30]:
    cells = []
    for b in order:
        v = agg[b][f] / cnt[b]
        d = v - agg[base][f] / cnt[base]
        cells.append(f"{v:8.1f}{d:+8.1f}" if b != base else f"{v:16.1f}")
    print(f"{f:44s} " + " ".join(cells))
