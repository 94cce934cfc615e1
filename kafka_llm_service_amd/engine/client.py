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
import queue
import threading
import time
from dataclasses import asdict
from typing import AsyncIterator

from kafka_llm_service_amd.engine.sequence import SamplingParams, StepOutput

log = logging.getLogger("kafka.engine")
HEARTBEAT_S = 1.0
_WARM = itertools.count()


SPILL_FACTOR = float(os.environ.get("KAFKA_DP_SPILL_FACTOR", "2.0"))
SPILL_MIN = int(os.environ.get("KAFKA_DP_SPILL_MIN", "48"))


class EngineUnavailable(RuntimeError):
    """No live engine can take the request (replica died / restarting / collective timeout): HTTP 503."""


def route(key: str | None, n: int, loads: list[int], alive: list[bool] | None = None,
          spill_factor: float = SPILL_FACTOR, spill_min: int = SPILL_MIN) -> int:
    """Replica for a request: the thread's home replica (stable hash of the thread id, so its KV prefix is reused);
    if that one is down, the next live replica in hash order; keyless requests go to the least-loaded live replica.
    Load-aware spill: when the home replica carries >= ``spill_min`` active requests AND more than ``spill_factor``
    x the mean live load, the request goes to the least-loaded live replica instead (a hot spot of threads costs one
    history re-prefill there — the shared system prefix is cached on every replica). Returns -1 when none is up."""
    live = [i for i in range(n) if alive is None or alive[i]]
    if not live:
        return -1
    least = min(live, key=lambda i: loads[i])
    if key is None:
        return least
    h = int(hashlib.blake2b(key.encode(), digest_size=8).hexdigest(), 16) % n
    home = -1
    for j in range(n):
        if alive is None or alive[(h + j) % n]:
            home = (h + j) % n
            break
    mean = sum(loads[i] for i in live) / len(live)
    if loads[home] >= spill_min and loads[home] > spill_factor * (mean + 1):
        return least
    return home


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

    def pin_prefix(self, token_ids: list[int]) -> None:
        self.async_engine.pin_prefix(token_ids)

    async def warm_prefix(self, token_ids: list[int]) -> None:
        """Prefill ``token_ids`` once (one sampled token, discarded) and pin the resulting pages."""
        sp = SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True)
        async for _ in self.async_engine.generate(f"warm-{next(_WARM)}", list(token_ids) + [0], sp):
            pass
        self.pin_prefix(token_ids)

    def health(self) -> dict:
        return {"replicas": 1, "replica0": self.async_engine.health()}

    async def close(self) -> None:
        self.async_engine.shutdown()


# ---------------------------------------------------------------------------------------------------------------
def _worker_main(rank: int, cfg_dict: dict, conn, n_local: int = 1) -> None:
    """One DP replica (tp = 1): owns one GPU, steps its engine, exchanges small pickled messages over a pipe."""
    from kafka_llm_service_amd.utils.affinity import pin_local_process

    pin_local_process(rank, n_local)
    from kafka_llm_service_amd.engine import fake

    fe = fake.from_env()  # KAFKA_FAKE_ENGINE_STEP_MS: timing-only engine (API-path load tests on the CPU)
    if fe is not None:
        conn.send(("ready", {"device": "fake", "kv_pages": 0}))
        serve_pipe(fe, conn)
        return
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
    """Request loop of a replica (or TP-group leader): drain control messages, step while there is work, send a
    heartbeat at least every HEARTBEAT_S (the parent's stall detector, ``DPClient._monitor``).
    ``KAFKA_ENGINE_PROFILE=<path>``: host-side cProfile of the loop, written when the replica is stopped."""
    path = os.environ.get("KAFKA_ENGINE_PROFILE")
    if not path:
        return _serve_pipe(eng, conn)
    import cProfile
    import pstats

    prof = cProfile.Profile()
    try:
        prof.runcall(_serve_pipe, eng, conn)
    finally:
        with open(f"{path}.{os.getpid()}", "w") as f:
            st = pstats.Stats(prof, stream=f)
            st.sort_stats("tottime").print_stats(50)
            st.sort_stats("cumtime").print_stats(70)


def _serve_pipe(eng, conn) -> None:
    from kafka_llm_service_amd.utils import faults

    from kafka_llm_service_amd.obs import trace

    fi = faults.get()
    tr = trace.tracer()
    pinned: list[int] | None = None  # the shared prefix; "add" messages may reference it instead of carrying it
    last_hb = 0.0
    while True:
        now = time.monotonic()
        if now - last_hb >= HEARTBEAT_S:
            conn.send(("hb", eng.stats["steps"]))
            last_hb = now
        if fi.worker_should_exit(eng.stats["steps"]):
            os._exit(3)  # injected replica crash (KAFKA_FI_WORKER_EXIT_AFTER)
        busy = eng.has_unfinished()
        while conn.poll(0 if busy else 0.05):
            msg = conn.recv()
            kind = msg[0]
            if kind == "add":
                _, rid, prompt, pdict, *sent = msg
                try:
                    if isinstance(prompt, tuple):  # ("ref", n, suffix): the first n ids are the pinned prefix
                        if pinned is None or len(pinned) < prompt[1]:
                            raise ValueError("prompt references a shared prefix this replica was not sent")
                        prompt = pinned[:prompt[1]] + prompt[2]
                    eng.add_request(rid, prompt, SamplingParams(**pdict))
                except Exception as e:
                    conn.send(("error", rid, str(e)))
                if sent and tr is not None:  # API submit -> engine admission (perf_counter is system-wide)
                    tr.complete("pipe_in", "engine", sent[0], time.perf_counter(), f"req:{rid}")
            elif kind == "abort":
                eng.abort(msg[1])
            elif kind == "pin":
                pinned = list(msg[1])
                eng.pin_prefix(pinned)
            elif kind == "health":
                kv = eng.kv_stats()
                conn.send(("health", {"running": eng.num_running, "waiting": eng.num_waiting,
                                      "kv_free_pages": kv["free"] + kv["evictable"],
                                      "kv_total_pages": kv["num_blocks"], "prefix_hit_tokens": kv["hit_tokens"],
                                      "output_tokens": eng.stats["output_tokens"], "steps": eng.stats["steps"],
                                      "perf": eng.perf_stats()}))
            elif kind == "stop":
                conn.send(("stopped",))
                return
            busy = eng.has_unfinished()
        if busy:
            outs = eng.step()
            if outs:
                conn.send(("out", [(o.request_id, o.new_token_ids, o.finished, o.finish_reason, o.num_prompt_tokens,
                                    o.num_output_tokens, o.num_cached_tokens) for o in outs], time.perf_counter()))


class DPClient:
    """``n_replicas`` independent engines; with ``tp > 1`` each replica is a TP group of ``tp`` processes
    (``engine/tp_worker.py``) whose leader owns the request pipe.

    Supervision (SURVEY.md §5.3 "engine watchdog ... the DP router drains and re-routes threads"): a replica whose
    process dies fails its in-flight streams with an error (the API turns it into an error frame), is marked down —
    its threads are routed to the next live replica and re-prefill from the thread store there — and is respawned in
    the background; a replica whose heartbeat stops for ``stall_timeout`` seconds is killed and handled the same way.
    """

    def __init__(self, engine_cfg, n_replicas: int, start_timeout: float = 900.0, tp: int = 1,
                 base_port: int | None = None, respawn: bool = True, stall_timeout: float | None = None,
                 dp_attention: bool = False):
        self._ctx = mp.get_context("spawn")
        self.engine_cfg = engine_cfg
        self.n_replicas = n_replicas
        self.tp = tp
        # Mixtral DP attention (engine/dp_attention.py): the replicas are the ranks of ONE EP group — each serves
        # its own threads (same thread-affinity routing), all of them step in lockstep and share the experts; the
        # group is spawned, and respawned, as a whole
        self.dpa = dp_attention
        if dp_attention and (tp != 1 or n_replicas < 2):
            raise ValueError("DP attention needs tp = 1 and at least 2 replicas")
        self._dpa_lock = threading.Lock()
        self.max_model_len = engine_cfg.max_model_len
        from kafka_llm_service_amd.models.config import get_config

        self.model_cfg = get_config(engine_cfg.model)
        self._cfg = asdict(engine_cfg)
        self._cfg["device"] = None
        self.start_timeout = start_timeout
        self.respawn = respawn
        self.stall_timeout = stall_timeout if stall_timeout is not None else \
            float(os.environ.get("KAFKA_STALL_TIMEOUT_S", "600"))
        self.conns: list = [None] * n_replicas
        self.procs: list = [None] * n_replicas
        self._group_procs: list[list] = [[] for _ in range(n_replicas)]
        self._send_locks = [threading.Lock() for _ in range(n_replicas)]
        # the request path's messages (add / abort) leave through one sender thread per replica: Connection.send
        # blocks once the pipe buffer is full, and the replica drains its pipe only between steps — a burst of new
        # turns sent from the event loop stalled the whole API for up to a step of a busy engine (175 ms measured,
        # profiles/r06/serve/). FIFO per replica keeps add -> abort order; tagged with the replica generation
        self._outq = [queue.SimpleQueue() for _ in range(n_replicas)]
        self._streams: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue, int]] = {}
        self._lock = threading.Lock()
        self._loads = [0] * n_replicas
        self._health: list[dict] = [{} for _ in range(n_replicas)]
        self._alive = [False] * n_replicas
        self._last_hb = [time.monotonic()] * n_replicas
        self._gen = [0] * n_replicas
        self.restarts = [0] * n_replicas
        self._closing = False
        self._ids = itertools.count()
        # the pinned shared prefix (~37k ids for the reference prompt): requests that start with it send only their
        # suffix over the pipe (pickling the full id list cost ~0.8 ms of API-loop time per request, serialized over
        # a burst of new turns) once the replica has been sent the prefix itself
        self._pin: list[int] | None = None
        self._pin_sent = [False] * n_replicas
        ports = base_port if base_port is not None else _free_port_base(n_replicas)
        self._dpa_port = ports  # DP attention: one rendezvous for the whole group
        pending = [self._spawn(r, ports + r) for r in range(n_replicas)]
        for r, conns in enumerate(pending):
            self._await_ready(r, conns)
        self._monitor_thread = threading.Thread(target=self._monitor, daemon=True, name="kafka-dp-monitor")
        self._monitor_thread.start()
        for r in range(n_replicas):
            threading.Thread(target=self._sender, args=(r,), daemon=True, name=f"kafka-dp-sender{r}").start()

    # ---- replica lifecycle -------------------------------------------------------------------------------------
    def _spawn(self, r: int, port: int) -> list:
        """Start replica r's processes; returns [leader_conn, follower_conns...] (not yet ready)."""
        ctx, cfg = self._ctx, self._cfg
        if self.dpa:
            from kafka_llm_service_amd.engine.dp_attention import dpa_worker_main

            parent, child = ctx.Pipe()
            p = ctx.Process(target=dpa_worker_main, args=(r, self.n_replicas, self._dpa_port, cfg, child),
                            daemon=True, name=f"kafka-dpa{r}")
            p.start()
            self.procs[r], self._group_procs[r] = p, [p]
            return [parent]
        if self.tp == 1:
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_worker_main, args=(r, cfg, child, self.n_replicas), daemon=True,
                            name=f"kafka-replica{r}")
            p.start()
            self.procs[r], self._group_procs[r] = p, [p]
            return [parent]
        from kafka_llm_service_amd.engine.tp_worker import tp_worker_main

        conns, group = [], []
        for t in range(self.tp):
            parent, child = ctx.Pipe()
            p = ctx.Process(target=tp_worker_main, args=(r, t, self.tp, port, cfg, child), daemon=True,
                            name=f"kafka-replica{r}-tp{t}")
            p.start()
            conns.append(parent)
            group.append(p)
        self.procs[r], self._group_procs[r] = group[0], group
        return conns

    def _await_ready(self, r: int, conns: list) -> None:
        deadline = time.monotonic() + self.start_timeout
        for c in conns:
            if not c.poll(max(1.0, deadline - time.monotonic())):
                raise RuntimeError(f"engine replica {r} did not start")
            msg = c.recv()
            if msg[0] != "ready":
                raise RuntimeError(f"engine replica {r} failed: {msg[1]}")
        with self._lock:
            self.conns[r] = conns[0]
            self._gen[r] += 1
            self._alive[r] = True
            self._last_hb[r] = time.monotonic()
            self._pin_sent[r] = False
        if self._pin is not None:  # a respawned replica learns the shared prefix again before any request
            self._send_quiet(r, ("pin", self._pin))
            self._pin_sent[r] = True
        threading.Thread(target=self._reader, args=(r, conns[0], self._gen[r]), daemon=True,
                         name=f"kafka-dp-reader{r}").start()

    def _respawn(self, r: int) -> None:
        if self.dpa:
            return self._respawn_dpa_group()
        for p in self._group_procs[r]:
            if p.is_alive():
                p.terminate()
            p.join(timeout=30)
        if self._closing or not self.respawn:
            return
        try:
            self._await_ready(r, self._spawn(r, _free_port_base(1)))
            self.restarts[r] += 1
            log.warning("engine replica %d restarted", r)
        except Exception:
            log.exception("engine replica %d failed to restart", r)

    def _respawn_dpa_group(self) -> None:
        """A DP-attention rank died: its peers cannot step without it, so the whole group is stopped, its streams
        failed (503 / error frames) and the group restarted on a fresh rendezvous (one thread does it; the other
        ranks' readers, which see their pipes close meanwhile, leave it to that one)."""
        if not self._dpa_lock.acquire(blocking=False):
            return
        try:
            for q in range(self.n_replicas):
                self._fail_replica(q)
                for p in self._group_procs[q]:
                    if p.is_alive():
                        p.kill()
                    p.join(timeout=30)
            if self._closing or not self.respawn:
                return
            self._dpa_port = _free_port_base(1)
            pending = [self._spawn(q, self._dpa_port) for q in range(self.n_replicas)]
            for q, conns in enumerate(pending):
                self._await_ready(q, conns)
                self.restarts[q] += 1
            log.warning("DP-attention group restarted")
        except Exception:
            log.exception("DP-attention group failed to restart")
        finally:
            self._dpa_lock.release()

    def _monitor(self) -> None:
        while not self._closing:
            time.sleep(1.0)
            now = time.monotonic()
            for r in range(self.n_replicas):
                if self._alive[r] and now - self._last_hb[r] > self.stall_timeout:
                    log.error("engine replica %d stalled (no heartbeat for %.0fs): killing it", r,
                              now - self._last_hb[r])
                    for p in self._group_procs[r]:
                        if p.is_alive():
                            p.kill()

    def _send(self, r: int, msg) -> None:
        with self._send_locks[r]:
            self.conns[r].send(msg)

    def _post(self, r: int, msg) -> None:
        """Queue msg for replica r's sender thread (never blocks the caller)."""
        self._outq[r].put((self._gen[r], msg))

    def _sender(self, r: int) -> None:
        while True:
            gen, msg = self._outq[r].get()
            if msg is None:
                return
            if gen != self._gen[r]:
                continue  # for a replica process that has been replaced: its streams were failed with it
            try:
                self._send(r, msg)
            except (OSError, BrokenPipeError, EOFError, AttributeError):
                if msg[0] == "add":  # the replica died between routing and this send: fail the stream now
                    with self._lock:
                        st = self._streams.pop(msg[1], None)
                        if st is not None:
                            self._loads[r] -= 1
                    if st is not None:
                        st[0].call_soon_threadsafe(st[1].put_nowait, EngineUnavailable(f"engine replica {r} is down"))

    def _send_quiet(self, r: int, msg) -> None:
        """Best-effort control message (aborts): a replica that is down has nothing to abort."""
        try:
            self._send(r, msg)
        except (OSError, BrokenPipeError, EOFError):
            pass

    def _reader(self, r: int, conn, gen: int) -> None:
        from kafka_llm_service_amd.obs import trace

        tr = trace.tracer()
        while True:
            try:
                msg = conn.recv()
            except (EOFError, OSError):
                if gen == self._gen[r] and not self._closing:
                    self._fail_replica(r)
                    threading.Thread(target=self._respawn, args=(r,), daemon=True).start()
                return
            kind = msg[0]
            if kind == "hb":
                self._last_hb[r] = time.monotonic()
            elif kind == "out":
                if tr is not None and len(msg) > 2 and any(o[5] == 1 for o in msg[1]):  # engine send -> reader
                    tr.complete("pipe_out", "api", msg[2], time.perf_counter(), f"replica{r}",
                                {"outs": len(msg[1])})
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
            self._alive[r] = False
            dead = [(rid, s) for rid, s in self._streams.items() if s[2] == r]
            for rid, _ in dead:
                self._streams.pop(rid, None)
            self._loads[r] = 0
        for rid, (loop, q, _) in dead:
            loop.call_soon_threadsafe(q.put_nowait, EngineUnavailable(f"engine replica {r} died"))

    async def generate(self, request_id: str, prompt_ids: list[int], params: SamplingParams,
                       routing_key: str | None = None) -> AsyncIterator[StepOutput]:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            r = route(routing_key, self.n_replicas, self._loads, self._alive)
            if r < 0:
                raise EngineUnavailable("no engine replica available (all replicas are restarting)")
            self._streams[request_id] = (loop, q, r)
            self._loads[r] += 1
        pd = {k: v for k, v in params.__dict__.items() if k != "allowed_tokens_fn"}
        pin = self._pin
        n = len(pin) if pin is not None and self._pin_sent[r] else 0
        if n and len(prompt_ids) > n and prompt_ids[n - 1] == pin[n - 1] and prompt_ids[:n] == pin:
            payload = ("ref", n, list(prompt_ids[n:]))
        else:
            payload = list(prompt_ids)
        self._post(r, ("add", request_id, payload, pd, time.perf_counter()))
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
                self._post(r, ("abort", request_id))

    def abort(self, request_id: str) -> None:
        with self._lock:
            s = self._streams.get(request_id)
        if s is not None:
            self._post(s[2], ("abort", request_id))

    async def warm_prefix(self, token_ids: list[int]) -> None:
        """Prefill the shared prefix on EVERY live replica (bypassing thread routing), then pin it everywhere."""
        loop = asyncio.get_running_loop()
        sp = {k: v for k, v in SamplingParams(temperature=0.0, max_tokens=1, ignore_eos=True).__dict__.items()
              if k != "allowed_tokens_fn"}
        waits = []
        for r in range(self.n_replicas):
            if not self._alive[r]:
                continue
            rid = f"warm-{next(_WARM)}-r{r}"
            q: asyncio.Queue = asyncio.Queue()
            with self._lock:
                self._streams[rid] = (loop, q, r)
                self._loads[r] += 1
            self._send(r, ("add", rid, list(token_ids) + [0], sp))
            waits.append(q)
        for q in waits:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    raise item
                if item.finished:
                    break
        self.pin_prefix(token_ids)

    def pin_prefix(self, token_ids: list[int]) -> None:
        """Every replica holds (and pins) its own copy of the shared system prefix."""
        self._pin = list(token_ids)
        for r in range(self.n_replicas):
            if self._alive[r]:
                self._send_quiet(r, ("pin", self._pin))
                self._pin_sent[r] = True

    def health(self) -> dict:
        for r in range(self.n_replicas):
            self._post(r, ("health",))  # (answered asynchronously: the reader stores it for the next call)
        out = {"replicas": self.n_replicas}
        for r in range(self.n_replicas):
            out[f"replica{r}"] = dict(self._health[r], active=self._loads[r], alive=bool(self._alive[r]),
                                      restarts=self.restarts[r])
        return out

    async def close(self) -> None:
        self._closing = True
        for r in range(self.n_replicas):
            self._outq[r].put((self._gen[r], None))  # stops the sender thread
        for r in range(self.n_replicas):
            try:
                self._send(r, ("stop",))
            except (OSError, BrokenPipeError, AttributeError):
                pass
        for group in self._group_procs:
            for p in group:
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
    if n == 1 and server_cfg.tp == 1 and not getattr(server_cfg, "engine_process", False):
        return await asyncio.to_thread(InProcessClient, ecfg)
    dpa = bool(getattr(server_cfg, "dp_attention", False))
    return await asyncio.to_thread(DPClient, ecfg, n, 900.0, max(1, server_cfg.tp), None, True, None, dpa)
