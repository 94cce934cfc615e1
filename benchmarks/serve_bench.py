#!/usr/bin/env python3
"""HTTP serving benchmark: concurrent multi-turn threads against ``POST /v1/threads/{id}/chat/completions``.

The load generator of SURVEY.md §4.4 ("BASELINE configs 1-5 with an OpenAI-SSE load generator: p50/p99 TTFT, TPOT,
output tok/s") and the method of the reference measurement in BASELINE.md §2 / SURVEY.md §6.2: a real uvicorn server
(1 worker) serving the app, an httpx async client, each thread runs ``--turns`` sequential turns, every turn is a new
user message on the thread (the server re-renders the whole history, so turns 2+ hit the prefix cache).

Reported (one JSON line): p50/p99 TTFT (first content frame, stream), p50/p99 end-to-end, TPOT, output tokens/s
(from the ``include_usage`` frame; the stub backend's 128 chunks count as 128 tokens), requests/s.

  # BASELINE config 1 (stub echo provider, CPU): compare with the reference's 3.9 ms p50 TTFT (1 thread) and
  # 190 ms p50 TTFT / 22.3k chunks/s (64 threads)
  python benchmarks/serve_bench.py --backend stub --threads 64 --turns 4
  # engine backend on one GPU (random-init Llama-3-8B, real Kafka system prompt):
  python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 --max-tokens 128
  # an already running server:
  python benchmarks/serve_bench.py --url http://127.0.0.1:8081 --threads 64
"""
from __future__ import annotations

import argparse
import functools
import asyncio
import json
import os
import socket
import statistics
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


async def _turn(client, url, tid, i, args, res):
    body = {"model": args.model_name, "stream": not args.no_stream, "max_tokens": args.max_tokens,
            "temperature": args.temperature, "messages": [{"role": "user", "content": f"turn {i} of thread {tid}: "
                                                                                        + "hello " * args.user_words}]}
    if not args.no_stream:
        body["stream_options"] = {"include_usage": True}
    t0 = time.perf_counter()
    ttft = None
    out_tok = 0
    if args.no_stream:
        r = await client.post(f"{url}/v1/threads/{tid}/chat/completions", json=body)
        j = r.json()
        out_tok = (j.get("usage") or {}).get("completion_tokens", 0)
    else:
        async with client.stream("POST", f"{url}/v1/threads/{tid}/chat/completions", json=body) as r:
            # cheap framing: only the first content frame (TTFT) and the usage frame are JSON-decoded, so the
            # client is not the bottleneck at 64 concurrent streams of 128 frames each
            buf = b""
            async for chunk in r.aiter_raw():
                buf += chunk
                if ttft is None and b'"content":"' in buf:
                    ttft = time.perf_counter() - t0
                *frames, buf = buf.split(b"\n\n")
                for frame in frames:
                    if b'"usage"' in frame or b'"error"' in frame:
                        d = json.loads(frame[6:])
                        if "error" in d:
                            raise RuntimeError(d["error"])
                        if d.get("usage"):
                            out_tok = d["usage"]["completion_tokens"]
    e2e = time.perf_counter() - t0
    res["e2e"].append(e2e)
    res.setdefault("by_turn", {}).setdefault(i, []).append(e2e)
    if ttft is not None:
        res["ttft"].append(ttft)
        res.setdefault("ttft_by_turn", {}).setdefault(i, []).append(ttft)
        if out_tok > 1:
            res["tpot"].append((e2e - ttft) / (out_tok - 1))
    res["tokens"] += out_tok
    res["requests"] += 1


_SYS_WORDS = ("tool shell notebook thread agent planner sandbox weather stream token cache prefix kernel wave "
              "matrix memory schedule request reply history playbook profile idle summary context").split()


@functools.lru_cache(maxsize=4)
def _system_message(chars: int) -> str | None:
    """A deterministic synthetic system prompt of ~``chars`` characters, identical for every thread (the reference's
    rendered Kafka prompt is ~70k characters; a thread created with a system message carries it as its prefix)."""
    if chars <= 0:
        return None
    out, i, n = [], 0, 0
    while n < chars:
        w = _SYS_WORDS[(i * 7 + i // 13) % len(_SYS_WORDS)]
        out.append(w)
        n += len(w) + 1
        i += 1
    return " ".join(out)


# The reference's 13 prompt sections (rendered: 70,496 characters) encode to 17,032 tokens with the engine's
# Llama-3-class BPE (engine/tokenizer.py, round 4; 18,151 with the server's tool schemas — the round-3 toy BPE made
# that 37.4k). ``--system-tokens ref`` serves a synthetic shared prefix of the reference prompt's size (+ schemas);
# ``--system-tokens 18000`` the headline bench's 18k shared prefix, so the API-path tax on the engine metric is
# measured like for like.
REFERENCE_PROMPT_TOKENS = 18151


@functools.lru_cache(maxsize=4)
def _system_message_tokens(n: int) -> str:
    """A synthetic system prompt of exactly ``n`` tokens under the engine's tokenizer."""
    from kafka_llm_service_amd.engine.tokenizer import get_tokenizer

    tok = get_tokenizer()
    text = _system_message(8 * n)
    ids = tok.encode(text)[:n]
    return tok.decode(ids)


async def _thread(client, url, k, args, res):
    if getattr(args, "stagger", 0) > 0 and k >= 0:
        # steady-state arrivals: thread k starts at a deterministic point in [0, stagger) instead of all at once
        await asyncio.sleep(args.stagger * ((k * 0.6180339887) % 1.0))
    if args.system_tokens:
        body = {"system_message": _system_message_tokens(args.system_tokens)}
    else:
        body = {"system_message": _system_message(args.system_chars)} if args.system_chars > 0 else {}
    r = await client.post(f"{url}/v1/threads", json=body)
    tid = r.json()["thread_id"]
    for i in range(args.turns):
        await _turn(client, url, tid, i, args, res)


async def _drive(url, args, k0, k1, warm):
    import httpx

    n = k1 - k0
    limits = httpx.Limits(max_connections=n + 8, max_keepalive_connections=n + 8)
    async with httpx.AsyncClient(timeout=httpx.Timeout(600.0), limits=limits) as client:
        for _ in range(300):
            try:
                if (await client.get(f"{url}/health")).json().get("kafka_initialized"):
                    break
            except Exception:
                pass
            await asyncio.sleep(1.0)
        if warm:  # one thread, one turn: fills the shared system-prompt prefix cache
            await _thread(client, url, -1, argparse.Namespace(**{**vars(args), "turns": 1}),
                          {"e2e": [], "ttft": [], "tpot": [], "tokens": 0, "requests": 0})
        res = {"e2e": [], "ttft": [], "tpot": [], "tokens": 0, "requests": 0}
        t0 = time.perf_counter()
        c0 = time.process_time()
        await asyncio.gather(*[_thread(client, url, k, args, res) for k in range(k0, k1)])
        res["wall"] = time.perf_counter() - t0
        res["client_cpu"] = time.process_time() - c0
    return res


def _proc_main(url, args, k0, k1, start_evt, q):
    start_evt.wait()
    q.put(asyncio.run(_drive(url, args, k0, k1, False)))


def run(url, args):
    """Drive ``args.threads`` threads from ``args.procs`` client processes (one httpx client saturates a core at
    ~250 streamed requests/s, which would make the LOAD GENERATOR the bottleneck); percentiles over all requests."""
    import multiprocessing as mp

    asyncio.run(_drive(url, argparse.Namespace(**{**vars(args), "turns": 1}), -1, -1, True))
    P = max(1, min(args.procs, args.threads))
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    start = ctx.Event()
    bounds = [(args.threads * i // P, args.threads * (i + 1) // P) for i in range(P)]
    procs = [ctx.Process(target=_proc_main, args=(url, args, a, b, start, q)) for a, b in bounds]
    for p in procs:
        p.start()
    time.sleep(0.5)
    t0 = time.perf_counter()
    start.set()
    parts = [q.get() for _ in procs]
    wall = time.perf_counter() - t0
    for p in procs:
        p.join()
    res = {"e2e": [], "ttft": [], "tpot": [], "tokens": 0, "requests": 0, "by_turn": {}, "client_cpu": 0.0}
    for r in parts:
        for k in ("e2e", "ttft", "tpot"):
            res[k] += r[k]
        res["tokens"] += r["tokens"]
        res["requests"] += r["requests"]
        res["client_cpu"] += r["client_cpu"]
        for t, v in r.get("by_turn", {}).items():
            res["by_turn"].setdefault(t, []).extend(v)
        for t, v in r.get("ttft_by_turn", {}).items():
            res.setdefault("ttft_by_turn", {}).setdefault(t, []).extend(v)
    ms = lambda v: None if v is None else round(v * 1e3, 2)  # noqa: E731
    return {
        "metric": "serve: p50 TTFT + output tok/s, /v1/threads/{id}/chat/completions",
        "backend": args.backend, "model": args.model, "threads": args.threads, "turns": args.turns,
        "stream": not args.no_stream, "client_procs": P, "system_chars": args.system_chars,
        "system_tokens": args.system_tokens,
        "stagger_s": args.stagger, "requests": res["requests"], "wall_s": round(wall, 3),
        "client_cpu_s": round(res["client_cpu"], 3),
        "ttft_p50_ms": ms(_pct(res["ttft"], 0.5)), "ttft_p99_ms": ms(_pct(res["ttft"], 0.99)),
        "e2e_p50_ms": ms(_pct(res["e2e"], 0.5)), "e2e_p99_ms": ms(_pct(res["e2e"], 0.99)),
        "tpot_p50_ms": ms(statistics.median(res["tpot"])) if res["tpot"] else None,
        "output_tok_s": round(res["tokens"] / wall, 1), "requests_s": round(res["requests"] / wall, 1),
        "e2e_p50_ms_by_turn": {k: ms(_pct(v, 0.5)) for k, v in sorted(res["by_turn"].items())},
        "ttft_p50_p99_ms_by_turn": {k: [ms(_pct(v, 0.5)), ms(_pct(v, 0.99))]
                                    for k, v in sorted(res.get("ttft_by_turn", {}).items())},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default=None, help="target an already running server instead of starting one")
    ap.add_argument("--backend", default="stub", choices=["stub", "engine"])
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--model-name", default="kafka")
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--threads", type=int, default=64)
    ap.add_argument("--turns", type=int, default=4)
    ap.add_argument("--stagger", type=float, default=0.0,
                    help="spread thread starts over this many seconds (0 = all threads start together, a burst)")
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--user-words", type=int, default=8)
    ap.add_argument("--no-stream", action="store_true")
    ap.add_argument("--procs", type=int, default=4, help="load-generator processes")
    ap.add_argument("--system-chars", type=int, default=0,
                    help="create threads with a shared synthetic system message of this many characters "
                         "(70000 ~ the reference's rendered Kafka prompt) instead of the server's Kafka prompt")
    ap.add_argument("--system-tokens", default=None,
                    help="shared synthetic system message of exactly this many engine tokens; 'ref' = the size of "
                         f"the reference's Kafka prompt ({REFERENCE_PROMPT_TOKENS} tokens)")
    ap.add_argument("--ignore-eos", action="store_true", default=True)
    args = ap.parse_args()
    if args.system_tokens is not None:
        args.system_tokens = REFERENCE_PROMPT_TOKENS if args.system_tokens == "ref" else int(args.system_tokens)
    proc = None
    url = args.url
    if url is None:
        port = _free_port()
        env = dict(os.environ, KAFKA_LLM_BACKEND=args.backend, KAFKA_MODEL=args.model, KAFKA_DP=str(args.dp),
                   KAFKA_TP=str(args.tp), KAFKA_SANDBOX="none", LOCAL_DB_PATH=":memory:",
                   KAFKA_IGNORE_EOS="1" if args.ignore_eos else "0", DEFAULT_MODEL=args.model_name,
                   PYTHONPATH=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        proc = subprocess.Popen([sys.executable, "-m", "kafka_llm_service_amd.server", "--host", "127.0.0.1",
                                 "--port", str(port)], env=env)
        url = f"http://127.0.0.1:{port}"
    try:
        out = run(url, args)
    finally:
        if proc is not None:
            proc.terminate()
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                proc.kill()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
