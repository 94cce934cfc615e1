#!/usr/bin/env python3
"""Per-request TTFT breakdown from KAFKA_TRACE_FILE traces of a serving run (Chrome trace JSON, one file per
process): p50 / p99 / mean of every API-side span (DB load, template render, submit -> first engine output, request
-> first SSE content frame) and of the engine's own arrival -> first-token span.

    python scripts/ttft_breakdown.py gpurun_out/trace.*.json
"""
import glob
import json
import statistics
import sys


def load(paths):
    evs = []
    for p in paths:  # one event per line (a process killed before closing its file leaves no trailing "]")
        for line in open(p):
            line = line.strip().rstrip(",")
            if line.startswith("{") and line.endswith("}") and line != "{}":
                try:
                    e = json.loads(line)
                except json.JSONDecodeError:
                    continue
                if e.get("ph") == "X":
                    evs.append(e)
    return evs


def main():
    paths = [q for a in sys.argv[1:] for q in glob.glob(a)]
    evs = load(paths)
    names = ["api_http_ttft", "api_db_load", "api_db_save", "api_render", "api_engine_first", "pipe_in", "first_token",
             "pipe_out"]

    def table(sel):
        print(f"{'span':20s} {'n':>6s} {'p50 ms':>9s} {'p99 ms':>9s} {'mean ms':>9s}")
        for n in names:
            d = sorted(e["dur"] / 1e3 for e in sel if e["name"] == n)
            if not d:
                continue
            print(f"{n:20s} {len(d):6d} {d[len(d) // 2]:9.2f} {d[min(len(d) - 1, int(0.99 * len(d)))]:9.2f} "
                  f"{statistics.fmean(d):9.2f}")
    table(evs)
    # the first burst: spans starting within 150 ms of the 8th request (every thread's first turn in a burst run;
    # a lone earlier request, e.g. a readiness probe, does not start it)
    starts = sorted(e["ts"] for e in evs if e["name"] == "api_http_ttft")
    t0 = starts[min(7, len(starts) - 1)] - 20e3 if starts else None
    if t0 is not None:
        print("-- request starts (ms after the first): " +
              " ".join(f"{(t - starts[0]) / 1e3:.0f}" for t in starts[:12]) + " ...")
        big = sorted(((e["dur"] / 1e3, (e["ts"] - starts[0]) / 1e3) for e in evs if e["name"] == "api_loop_lag"),
                     reverse=True)[:6]
        print("-- longest loop stalls (ms, at ms after the first request): " +
              ", ".join(f"{d:.0f} @ {t:.0f}" for d, t in big))
        gcs = sorted(((e["dur"] / 1e3, (e["ts"] - starts[0]) / 1e3, e["name"]) for e in evs
                      if e["name"].startswith("gc_gen")), reverse=True)
        if gcs:
            print(f"-- cyclic GC: {len(gcs)} collections, {sum(g[0] for g in gcs):.1f} ms; longest: " +
                  ", ".join(f"{n} {d:.1f} @ {t:.0f}" for d, t, n in gcs[:5]))
        first = [e for e in evs if t0 <= e["ts"] <= t0 + 150e3]
        print("-- first burst (spans starting within 150 ms of the first request)")
        table(first)
        lag0 = [e["dur"] / 1e3 for e in evs if e["name"] == "api_loop_lag" and t0 - 50e3 <= e["ts"] <= t0 + 400e3]
        print(f"   api loop lag in [-50, +400] ms: {len(lag0)} stalls, {sum(lag0):.1f} ms, longest "
              f"{max(lag0, default=0.0):.1f} ms")
    lag = sorted((e["ts"] / 1e3, e["dur"] / 1e3) for e in evs if e["name"] == "api_loop_lag")
    if lag:  # API event loop blocked (> 2 ms late wake-ups): total, longest, and the busiest 100 ms window
        tot = sum(d for _, d in lag)
        best, j = 0.0, 0
        for i in range(len(lag)):
            while lag[i][0] - lag[j][0] > 100.0:
                j += 1
            best = max(best, sum(d for _, d in lag[j:i + 1]))
        print(f"api loop lag: {len(lag)} stalls > 2 ms, {tot:.1f} ms in all, longest {max(d for _, d in lag):.1f} ms, "
              f"busiest 100 ms window {best:.1f} ms blocked")
    steps = sorted(e["dur"] / 1e3 for e in evs if e["name"] == "launch")
    if steps:
        print(f"engine launch spans: {len(steps)}, p50 {steps[len(steps) // 2]:.2f} ms")


if __name__ == "__main__":
    main()
