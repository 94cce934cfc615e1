"""Prometheus metrics: request counts, TTFT / end-to-end latency histograms, engine gauges
(running / waiting sequences, KV pages used / free, prefix-cache hit tokens, output tokens) scraped from the engine
client at render time, and per-GPU step time (``kafka_gpu_step_ms{replica,device,stat}``) and collective time
(``kafka_gpu_collective_ms_per_step``: the custom all-reduce / all-to-all kernels' own clock stamps, hipGraph
replays included). The reference exposed only /health (server.py:617-620)."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Histogram, generate_latest

REGISTRY = CollectorRegistry(auto_describe=True)
_BUCKETS = (0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5, 1.0, 2.0, 5.0, 10.0, 30.0, 60.0)
REQUESTS = Counter("kafka_requests_total", "HTTP requests by route", ["route"], registry=REGISTRY)
TTFT = Histogram("kafka_ttft_seconds", "time to first streamed content token", buckets=_BUCKETS, registry=REGISTRY)
E2E = Histogram("kafka_request_seconds", "end-to-end streamed request latency", buckets=_BUCKETS, registry=REGISTRY)
TPOT = Histogram("kafka_tpot_seconds", "time per output token after the first (streamed requests)",
                 buckets=(0.001, 0.002, 0.005, 0.01, 0.02, 0.05, 0.1, 0.2, 0.5), registry=REGISTRY)
OUTPUT_TOKENS = Counter("kafka_output_tokens_total", "generated tokens returned to clients", registry=REGISTRY)
TOOL_SECONDS = Histogram("kafka_tool_seconds", "tool execution time by tool", ["tool"], buckets=_BUCKETS,
                         registry=REGISTRY)


_PERF = {"step_ms_mean": ("kafka_gpu_step_ms", 'stat="mean"'), "step_ms_p50": ("kafka_gpu_step_ms", 'stat="p50"'),
         "step_ms_p99": ("kafka_gpu_step_ms", 'stat="p99"'),
         "collective_ms_per_step": ("kafka_gpu_collective_ms_per_step", ""),
         "collective_us_per_call": ("kafka_gpu_collective_us_per_call", ""),
         "collective_calls_per_step": ("kafka_gpu_collective_calls_per_step", "")}


def render(state) -> str:
    out = generate_latest(REGISTRY).decode()
    health = state.engine_health() if state is not None else {}
    lines = []
    for k, v in sorted(_flatten(health).items()):
        if isinstance(v, (int, float)) and not isinstance(v, bool):
            lines.append(f"kafka_engine_{k} {v}")
    # per-GPU step time and collective time, labelled by replica and device
    for rk, rv in sorted((health or {}).items()):
        perf = rv.get("perf") if isinstance(rv, dict) else None
        if not isinstance(perf, dict) or not rk.startswith("replica"):
            continue
        base = f'replica="{rk[len("replica"):]}",device="{perf.get("device", "")}"'
        for key, (name, extra) in _PERF.items():
            if isinstance(perf.get(key), (int, float)):
                lab = base + ("," + extra if extra else "")
                lines.append(f"{name}{{{lab}}} {perf[key]}")
    return out + "\n".join(lines) + ("\n" if lines else "")


def _flatten(d, prefix=""):
    out = {}
    for k, v in (d or {}).items():
        key = f"{prefix}{k}".replace(".", "_").replace("-", "_")
        if isinstance(v, dict):
            out.update(_flatten(v, key + "_"))
        else:
            out[key] = v
    return out
