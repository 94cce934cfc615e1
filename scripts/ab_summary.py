"""One line per run of a gpu_ab_env.sh A/B (gpurun_out/ab.jsonl): variant, round, tok/s, in-step GPU ms, p50 / p99
TTFT and the step-rows histogram; then the mean tok/s per variant. Usage: ab_summary.py ab.jsonl"""
import json
import statistics
import sys
from collections import defaultdict

runs = [json.loads(line) for line in open(sys.argv[1]) if line.startswith("{")]
per = defaultdict(list)
for d in runs:
    g = (d.get("gpu_ms_per_step") or {}).get("in_step")
    print(f"{d['variant']:12s} r{d.get('round', '?')}  {d['value']:9.1f} tok/s  in-step {g} ms  "
          f"TTFT p50 {d.get('ttft_p50_ms')} p99 {d.get('ttft_p99_ms')}  rows {d.get('step_rows_hist')}")
    per[d["variant"]].append(d["value"])
for v, xs in per.items():
    print(f"{v:12s} mean {statistics.fmean(xs):9.1f} tok/s over {len(xs)} runs ({min(xs):.1f} .. {max(xs):.1f})")
