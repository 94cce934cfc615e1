"""Summarise a rocprofv3 kernel_stats.csv: short name, calls, total ms, avg us, %."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':70s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for r in rows[:n]:
    name = r["Name"]
    name = re.sub(r"\(.*", "", name)
    name = name[:70]
    print(f"{name:70s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:10.2f} {float(r['AverageNs'])/1e3:9.1f} {float(r['Percentage']):6.2f}")
print(f"total kernel time {tot/1e6:.1f} ms")
