#!/usr/bin/env python3
"""BASELINE config 4 at its real size on ONE MI355X: Llama-3-70B (tiled-only weights, TP = 1: the 140 GB model and
its KV pool fit one GPU's 288 GB) serving /v1/threads/{id}/agent/run with the served default system prompt (the
reference's 13 sections + the server's tool schemas, ~18k tokens) and the working tool chain of tests/config4_flow.py
(create_shell -> shell_exec `ls` in the shipped sandbox service -> get_weather). Writes the SSE transcript and a
summary (per-iteration engine usage: prompt / cached tokens, wall time per LLM call) under --out.
TP = 8 over xGMI is the driver's 8-GPU run; this is the same agent loop on the model's real shapes and prompt.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--out", default="gpurun_out/config4_real")
    ap.add_argument("--max-model-len", type=int, default=32768)
    args = ap.parse_args()
    import config4_flow

    out = Path(args.out)
    out.mkdir(parents=True, exist_ok=True)
    t0 = time.perf_counter()
    metrics = {}

    def grab(c):
        metrics["text"] = c.get("/metrics").text

    with tempfile.TemporaryDirectory() as td:
        text, frames, msgs = config4_flow.run(Path(td), args.model, {}, sections=None, on_done=grab,
                                              max_model_len=args.max_model_len)
    (out / "metrics.txt").write_text(metrics.get("text", ""))
    wall = time.perf_counter() - t0
    (out / "agent_run_sse.txt").write_text(text)
    usage = [f for f in frames if f.get("type") == "usage"]
    calls = [tc["function"]["name"] for f in frames for ch in (f.get("choices") or [])
             for tc in (ch["delta"].get("tool_calls") or []) if (tc.get("function") or {}).get("name")]
    res = {f["tool_name"]: "" for f in frames if f.get("type") == "tool_result"}
    for f in frames:
        if f.get("type") == "tool_result":
            res[f["tool_name"]] += f["delta"]
    summary = {"model": args.model, "wall_s_incl_load": round(wall, 1), "tool_calls": calls,
               "usage": [u.get("usage") for u in usage], "iterations": [u.get("iteration") for u in usage],
               "tool_results": {k: v[:300] for k, v in res.items()},
               "roles": [m["role"] for m in msgs]}
    try:
        config4_flow.check(text, frames, msgs)
        summary["check"] = "pass"
    except AssertionError as e:  # recorded, and the exit code says so
        summary["check"] = f"FAIL: {e}"
    (out / "summary.json").write_text(json.dumps(summary, indent=1))
    print(json.dumps(summary)[:3000])
    return 0 if summary["check"] == "pass" else 1


if __name__ == "__main__":
    sys.exit(main())
