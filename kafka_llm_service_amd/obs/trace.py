"""Tracing ("per-request spans (queue -> prefill -> first token -> decode -> tool time) ... roctx
ranges around scheduler phases"). The reference had only print() calls.

* ``KAFKA_TRACE_FILE=/path/trace`` — every process writes Chrome trace-event JSON to ``/path/trace.<pid>.json``
  (open in chrome://tracing or Perfetto): engine step phases (schedule / plan / launch / collect / outputs), one span
  per request (queued -> first token -> finished, with prompt / cached / output token counts), agent LLM turns and
  tool executions.
* ``KAFKA_ROCTX=1`` — the same spans also open roctx ranges (``torch.cuda.nvtx`` lowers to roctx on ROCm), so a
  ``rocprofv3 --marker-trace`` run shows the scheduler phases on the timeline next to the kernels.
Both are off by default and cost one ``None`` check per span when off.
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager

_T0 = time.perf_counter()


class Tracer:
    def __init__(self, path: str):
        self.path = path
        self._f = open(path, "w")
        self._f.write("[\n")
        self._lock = threading.Lock()
        self._pid = os.getpid()
        self._last_flush = time.perf_counter()

    def complete(self, name: str, cat: str, start: float, end: float, tid: int | str | None = None,
                 args: dict | None = None) -> None:
        """A finished span; ``start``/``end`` are time.perf_counter() values."""
        ev = {"name": name, "cat": cat, "ph": "X", "ts": round((start - _T0) * 1e6, 1),
              "dur": round(max(0.0, end - start) * 1e6, 1), "pid": self._pid,
              "tid": tid if tid is not None else threading.get_ident()}
        if args:
            ev["args"] = args
        line = json.dumps(ev) + ",\n"
        with self._lock:
            self._f.write(line)
            now = time.perf_counter()
            if now - self._last_flush > 0.5:  # a process killed without exit handlers keeps all but the last 0.5 s
                self._f.flush()
                self._last_flush = now

    def flush(self) -> None:
        with self._lock:
            self._f.flush()

    def close(self) -> None:
        with self._lock:
            if not self._f.closed:
                self._f.write("{}]\n")
                self._f.close()


_TRACER: Tracer | None = None
_INIT = False
_ROCTX = None


def tracer() -> Tracer | None:
    global _TRACER, _INIT
    if not _INIT:
        _INIT = True
        base = os.environ.get("KAFKA_TRACE_FILE")
        if base:
            _TRACER = Tracer(f"{base}.{os.getpid()}.json")
            import atexit

            atexit.register(_TRACER.close)
    return _TRACER


def _roctx():
    global _ROCTX
    if _ROCTX is None:
        _ROCTX = False
        if os.environ.get("KAFKA_ROCTX") == "1":
            try:
                import torch

                if torch.cuda.is_available():
                    _ROCTX = torch.cuda.nvtx
            except Exception:
                _ROCTX = False
    return _ROCTX


@contextmanager
def span(name: str, cat: str = "engine", tid: int | str | None = None, **args):
    t = tracer()
    rx = _roctx()
    if t is None and not rx:
        yield
        return
    if rx:
        rx.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if rx:
            rx.range_pop()
        if t is not None:
            t.complete(name, cat, t0, time.perf_counter(), tid, args or None)


def request_span(seq, end: float) -> None:
    """One span per finished engine request (arrival -> finish) with its phase boundaries as args."""
    t = tracer()
    if t is None:
        return
    args = {"prompt_tokens": len(seq.prompt_ids), "cached_tokens": seq.num_cached,
            "output_tokens": len(seq.output_ids), "finish": seq.finish_reason, "preemptions": seq.preemptions}
    if seq.first_token_time is not None:
        args["ttft_ms"] = round((seq.first_token_time - seq.arrival) * 1e3, 3)
        t.complete("first_token", "request", seq.arrival, seq.first_token_time, f"req:{seq.request_id}")
        t.complete("decode", "request", seq.first_token_time, end, f"req:{seq.request_id}")
    t.complete("request", "request", seq.arrival, end, f"req:{seq.request_id}", args)
