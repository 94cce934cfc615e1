#!/usr/bin/env python3
"""Minimal client of a running server: creates a thread and streams two turns from
``/v1/threads/{id}/chat/completions`` the way an OpenAI SDK loop consumes them (``choices[0].delta.content``).

  python -m kafka_llm_service_amd.server &          # or KAFKA_LLM_BACKEND=stub for the echo backend
  python examples/client.py --url http://127.0.0.1:8081
"""
from __future__ import annotations

import argparse
import json

import httpx


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://127.0.0.1:8081")
    ap.add_argument("--model", default="kafka")
    a = ap.parse_args()
    with httpx.Client(base_url=a.url, timeout=600) as c:
        tid = c.post("/v1/threads", json={}).json()["thread_id"]
        for text in ("Hi! What can you do?", "Summarise that in one line."):
            print(f"\nuser: {text}\nassistant: ", end="", flush=True)
            body = {"model": a.model, "stream": True, "max_tokens": 64,
                    "messages": [{"role": "user", "content": text}], "stream_options": {"include_usage": True}}
            with c.stream("POST", f"/v1/threads/{tid}/chat/completions", json=body) as r:
                for line in r.iter_lines():
                    if not line.startswith("data: ") or line == "data: [DONE]":
                        continue
                    chunk = json.loads(line[6:])
                    if chunk.get("usage"):
                        print(f"\n[usage] {chunk['usage']}")
                    elif chunk.get("choices") and chunk["choices"][0]["delta"].get("content"):
                        print(chunk["choices"][0]["delta"]["content"], end="", flush=True)
        print("\nhistory:", [m["role"] for m in c.get(f"/v1/threads/{tid}/messages").json()["messages"]])


if __name__ == "__main__":
    main()
