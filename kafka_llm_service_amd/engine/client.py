"""Engine clients used by the API server: in-process (one GPU) or data-parallel worker processes (one per GPU).

DP serving (SURVEY.md §2.4 "DP replicas with thread affinity"): every replica is an independent engine with its own KV
cache on its own GPU. Requests are routed by a stable hash of the thread id, so all turns (and agent iterations) of
one thread land on the replica that already holds that thread's KV prefix; each replica holds its own copy of the
shared system-prompt prefix. Requests without a routing key go to the least-loaded replica. Replicas never talk to
each other on the hot path (no collectives), which is why the 8B configuration scales near-linearly over xGMI-
connected GPUs. Worker processes are started with the ``spawn`` method (each initialises its own HIP context).
"""
from __future__ import annotations

import asyncio
import hashlib
import itertools
import logging
import multiprocessing as mp
import os
import threading
import time
from dataclasses import asdict
from typing import AsyncIterator

from kafka_llm_service_amd.engine.sequence import SamplingParams, StepOutput

log = logging.getLogger("kafka.engine")


def route(key: str | None, n: int, loads: list[int]) -> int:
    if n == 1:
        return 0
    if key is None:
        return min(range(n), key=lambda i: loads[i])
    return int(hashlib.blake2b(key.encode(), digest_size=8).hexdigest(), 16) % n


class InProcessClient:
    def __init__(self, engine_cfg):
        from kafka_llm_service_amd.engine.async_engine import AsyncEngine
        from kafka_llm_service_amd.engine.engine import LLMEngine

        self.engine_cfg = engine_cfg
        self.async_engine = AsyncEngine(lambda: LLMEngine(engine_cfg))
        self.async_engine.start()
        eng = self.async_engine.engine
        self.model_cfg = eng.model_cfg
        self.max_model_len = engine_cfg.max_model_len
        self.n_replicas = 1

    async def generate(self, request_id: str, prompt_ids: list[int], params: SamplingParams,
                       routing_key: str | None = None) -> AsyncIterator[StepOutput]:
        async for o in self.async_engine.generate(request_id, prompt_ids, params):
            yield o

    def abort(self, request_id: str) -> None:
        self.async_engine.abort(request_id)

    def health(self) -> dict:
        return {"replicas": 1, "replica0": self.async_engine.health()}

    async def close(self) -> None:
        self.async_engine.shutdown()


# ---------------------------------------------------------------------------------------------------------------
def _worker_main(rank: int, cfg_dict: dict, conn) -> None:
    """One DP replica (tp = 1): owns one GPU, steps its engine, exchanges small pickled messages over a pipe."""
    import torch

    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine

    cfg = EngineConfig(**cfg_dict)
    if torch.cuda.is_available():
        cfg.device = f"cuda:{rank % torch.cuda.device_count()}"
    try:
        eng = LLMEngine(cfg)
    except BaseException as e:
        conn.send(("fatal", repr(e)))
        return
    conn.send(("ready", {"device": str(eng.device), "kv_pages": eng.num_blocks}))
    serve_pipe(eng, conn)


def serve_pipe(eng, conn) -> None:
    """Request loop of a replica (or TP-group leader): drain control messages, step while there is work."""
    while True:
        busy = eng.has_unfinished()
        while conn.poll(0 if busy else 0.05):
            msg = conn.recv()
            kind = msg[0]
            if kind == "add":
                _, rid, prompt, pdict = msg
                try:
                    eng.add_request(rid, prompt, SamplingParams(**pdict))
                except Exception as e:
                    conn.send(("error", rid, str(e)))
            elif kind == "abort":
                eng.abort(msg[1])
            elif kind == "health":
                kv = eng.kv_stats()
                conn.send(("health", {"running": eng.num_running, "waiting": eng.num_waiting,
                                      "kv_free_pages": kv["free"] + kv["evictable"],
                                      "kv_total_pages": kv["num_blocks"], "prefix_hit_tokens": kv["hit_tokens"],
                                      "output_tokens": eng.stats["output_tokens"], "steps": eng.stats["steps"]}))
            elif kind == "stop":
                conn.send(("stopped",))
                return
            busy = eng.has_unfinished()
        if busy:
            outs = eng.step()
            if outs:
                conn.send(("out", [(o.request_id, o.new_token_ids, o.finished, o.finish_reason, o.num_prompt_tokens,
                                    o.num_output_tokens, o.num_cached_tokens) for o in outs]))


class DPClient:
    """``n_replicas`` independent engines; with ``tp > 1`` each replica is a TP group of ``tp`` processes
    (``engine/tp_worker.py``) whose leader owns the request pipe."""

    def __init__(self, engine_cfg, n_replicas: int, start_timeout: float = 900.0, tp: int = 1,
                 base_port: int | None = None):
        ctx = mp.get_context("spawn")
        self.engine_cfg = engine_cfg
        self.n_replicas = n_replicas
        self.tp = tp
        self.max_model_len = engine_cfg.max_model_len
        from kafka_llm_service_amd.models.config import get_config

        self.model_cfg = get_config(engine_cfg.model)
        cfg = asdict(engine_cfg)
        cfg["device"] = None
        self.conns, self.procs = [], []
        self._followers: list = []
        self._send_locks = [threading.Lock() for _ in range(n_replicas)]
        self._streams: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue, int]] = {}
        self._lock = threading.Lock()
        self._loads = [0] * n_replicas
        self._health: list[dict] = [{} for _ in range(n_replicas)]
        self._ids = itertools.count()
        follower_conns = []
        if base_port is None:
            base_port = _free_port_base(n_replicas)
        for r in range(n_replicas):
            if tp == 1:
                parent, child = ctx.Pipe()
                p = ctx.Process(target=_worker_main, args=(r, cfg, child), daemon=True, name=f"kafka-replica{r}")
                p.start()
                self.conns.append(parent)
                self.procs.append(p)
                continue
            from kafka_llm_service_amd.engine.tp_worker import tp_worker_main

            for t in range(tp):
                parent, child = ctx.Pipe()
                p = ctx.Process(target=tp_worker_main, args=(r, t, tp, base_port + r, cfg, child), daemon=True,
                                name=f"kafka-replica{r}-tp{t}")
                p.start()
                (self.conns if t == 0 else follower_conns).append(parent)
                (self.procs if t == 0 else self._followers).append(p)
        deadline = time.monotonic() + start_timeout
        for r, c in enumerate(self.conns + follower_conns):
            if not c.poll(max(1.0, deadline - time.monotonic())):
                raise RuntimeError(f"engine process {r} did not start")
            msg = c.recv()
            if msg[0] != "ready":
                raise RuntimeError(f"engine process {r} failed: {msg[1]}")
        self._readers = [threading.Thread(target=self._reader, args=(r,), daemon=True) for r in range(n_replicas)]
        for t in self._readers:
            t.start()

    def _send(self, r: int, msg) -> None:
        with self._send_locks[r]:
            self.conns[r].send(msg)

    def _reader(self, r: int) -> None:
        conn = self.conns[r]
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                self._fail_replica(r)
                return
            kind = msg[0]
            if kind == "out":
                batches: dict = {}
                with self._lock:
                    for rid, toks, fin, reason, npt, nout, ncached in msg[1]:
                        s = self._streams.get(rid)
                        if s is None:
                            continue
                        batches.setdefault(s[0], []).append(
                            (s[1], StepOutput(rid, toks, fin, reason, npt, nout, ncached)))
                        if fin:
                            self._streams.pop(rid, None)
                            self._loads[r] -= 1
                for loop, items in batches.items():
                    loop.call_soon_threadsafe(_put_all, items)
            elif kind == "error":
                with self._lock:
                    s = self._streams.pop(msg[1], None)
                    if s:
                        self._loads[r] -= 1
                if s:
                    s[0].call_soon_threadsafe(s[1].put_nowait, ValueError(msg[2]))
            elif kind == "health":
                self._health[r] = msg[1]
            elif kind == "stopped":
                return

    def _fail_replica(self, r: int) -> None:
        with self._lock:
            dead = [(rid, s) for rid, s in self._streams.items() if s[2] == r]
            for rid, _ in dead:
                self._streams.pop(rid, None)
        for rid, (loop, q, _) in dead:
            loop.call_soon_threadsafe(q.put_nowait, RuntimeError(f"engine replica {r} died"))

    async def generate(self, request_id: str, prompt_ids: list[int], params: SamplingParams,
                       routing_key: str | None = None) -> AsyncIterator[StepOutput]:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            r = route(routing_key, self.n_replicas, self._loads)
            self._streams[request_id] = (loop, q, r)
            self._loads[r] += 1
        pd = {k: v for k, v in params.__dict__.items() if k != "allowed_tokens_fn"}
        self._send(r, ("add", request_id, list(prompt_ids), pd))
        done = False
        try:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    raise item
                yield item
                if item.finished:
                    done = True
                    return
        finally:
            if not done:
                with self._lock:
                    if self._streams.pop(request_id, None) is not None:
                        self._loads[r] -= 1
                self._send(r, ("abort", request_id))

    def abort(self, request_id: str) -> None:
        with self._lock:
            s = self._streams.get(request_id)
        if s is not None:
            self._send(s[2], ("abort", request_id))

    def health(self) -> dict:
        for r in range(self.n_replicas):
            try:
                self._send(r, ("health",))
            except (OSError, BrokenPipeError):
                pass
        out = {"replicas": self.n_replicas}
        for r in range(self.n_replicas):
            out[f"replica{r}"] = dict(self._health[r], active=self._loads[r], alive=self.procs[r].is_alive())
        return out

    async def close(self) -> None:
        for r in range(self.n_replicas):
            try:
                self._send(r, ("stop",))
            except (OSError, BrokenPipeError):
                pass
        for p in self.procs + self._followers:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()


def _free_port_base(n: int) -> int:
    """A base port with n free consecutive ports on 127.0.0.1 (one rendezvous per TP replica)."""
    import socket

    for _ in range(64):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            base = sk.getsockname()[1]
        if base + n >= 65535:
            continue
        ok = True
        for i in range(1, n):
            with socket.socket() as sk:
                try:
                    sk.bind(("127.0.0.1", base + i))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free port range")


def _put_all(items) -> None:
    for q, o in items:
        q.put_nowait(o)


async def make_engine_client(server_cfg):
    """Build the engine client for a ServerConfig (runs the blocking start-up off the event loop)."""
    from kafka_llm_service_amd.engine.engine import EngineConfig

    ecfg = EngineConfig(model=server_cfg.model, weights=server_cfg.weights, max_model_len=server_cfg.max_model_len,
                        **server_cfg.engine_kwargs)
    n = max(1, server_cfg.dp)
    if n == 1 and server_cfg.tp == 1:
        return await asyncio.to_thread(InProcessClient, ecfg)
    return await asyncio.to_thread(DPClient, ecfg, n, 900.0, max(1, server_cfg.tp))
