"""AsyncEngine: runs LLMEngine.step() on a dedicated driver thread and streams outputs to asyncio consumers.

The reference ran everything on one asyncio loop and its plumbing alone saturated at ~150-230
req/s (§6.2). Here the API loop only enqueues requests and receives per-step output batches: the driver thread owns
the engine (single writer of all KV/scheduler state), pulls new requests / aborts at every iteration boundary, and
delivers each step's outputs with ONE ``call_soon_threadsafe`` per consumer loop (not one per token).
"""
from __future__ import annotations

import asyncio
import logging
import queue
import threading
import time
from collections import defaultdict
from typing import AsyncIterator

from kafka_llm_service_amd.engine.sequence import SamplingParams, StepOutput

log = logging.getLogger("kafka.engine")


class AsyncEngine:
    def __init__(self, engine_factory, name: str = "engine0"):
        self._factory = engine_factory
        self.engine = None
        self.name = name
        self._inbox: queue.Queue = queue.Queue()
        self._streams: dict[str, tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._lock = threading.Lock()
        self._thread: threading.Thread | None = None
        self._stop = threading.Event()
        self._ready = threading.Event()
        self.error: BaseException | None = None
        self.stats = {"steps": 0, "busy_s": 0.0, "requests": 0}

    def start(self, wait: bool = True) -> None:
        self._thread = threading.Thread(target=self._run, name=f"kafka-{self.name}", daemon=True)
        self._thread.start()
        if wait:
            self._ready.wait()
            if self.error:
                raise RuntimeError(f"engine failed to start: {self.error}")

    def _run(self) -> None:
        try:
            self.engine = self._factory()
        except BaseException as e:  # surfaced by start()
            self.error = e
            self._ready.set()
            return
        self._ready.set()
        eng = self.engine
        while not self._stop.is_set():
            self._drain(block=not eng.has_unfinished())
            if not eng.has_unfinished():
                continue
            t0 = time.perf_counter()
            try:
                outs = eng.step()
            except BaseException as e:  # fail every in-flight request, keep serving new ones
                log.exception("engine step failed")
                self._fail_all(e)
                continue
            self.stats["steps"] += 1
            self.stats["busy_s"] += time.perf_counter() - t0
            if outs:
                self._deliver(outs)

    def _drain(self, block: bool) -> None:
        try:
            item = self._inbox.get(timeout=0.05) if block else self._inbox.get_nowait()
        except queue.Empty:
            return
        while True:
            kind = item[0]
            if kind == "add":
                _, rid, prompt, params, meta = item
                try:
                    self.engine.add_request(rid, prompt, params, meta)
                except Exception as e:  # context length etc. -> error to that stream only
                    self._deliver_error(rid, e)
            elif kind == "abort":
                self.engine.abort(item[1])
            elif kind == "pin":
                self.engine.pin_prefix(item[1])
            try:
                item = self._inbox.get_nowait()
            except queue.Empty:
                return

    def _deliver(self, outs: list[StepOutput]) -> None:
        by_loop: dict[asyncio.AbstractEventLoop, list] = defaultdict(list)
        with self._lock:
            for o in outs:
                s = self._streams.get(o.request_id)
                if s is None:
                    continue
                by_loop[s[0]].append((s[1], o))
                if o.finished:
                    self._streams.pop(o.request_id, None)
        for loop, items in by_loop.items():
            loop.call_soon_threadsafe(_put_all, items)

    def _deliver_error(self, rid: str, e: BaseException) -> None:
        with self._lock:
            s = self._streams.pop(rid, None)
        if s is not None:
            s[0].call_soon_threadsafe(s[1].put_nowait, e)

    def _fail_all(self, e: BaseException) -> None:
        with self._lock:
            streams, self._streams = self._streams, {}
        for rid, (loop, q) in streams.items():
            loop.call_soon_threadsafe(q.put_nowait, e)
            self._inbox.put(("abort", rid))

    # --- consumer API -----------------------------------------------------------------------------------------
    async def generate(self, request_id: str, prompt_ids: list[int], params: SamplingParams,
                       meta: dict | None = None) -> AsyncIterator[StepOutput]:
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        with self._lock:
            self._streams[request_id] = (loop, q)
        self.stats["requests"] += 1
        self._inbox.put(("add", request_id, prompt_ids, params, meta))
        finished = False
        try:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    raise item
                if not item.finished and not q.empty():
                    item = _merge(item, q)  # the loop fell behind: hand on every landed token in one event
                    if isinstance(item, BaseException):
                        raise item
                yield item
                if item.finished:
                    finished = True
                    return
        finally:
            if not finished:  # consumer went away (client disconnect): free the sequence and its KV
                with self._lock:
                    self._streams.pop(request_id, None)
                self._inbox.put(("abort", request_id))

    def abort(self, request_id: str) -> None:
        self._inbox.put(("abort", request_id))

    def pin_prefix(self, token_ids: list[int]) -> None:
        """Pin the cached pages of a hot shared prefix (applied on the driver thread, the single KV writer)."""
        self._inbox.put(("pin", list(token_ids)))

    def health(self) -> dict:
        eng = self.engine
        if eng is None:
            return {"ready": False}
        kv = eng.kv_stats()
        return {"ready": True, "running": eng.num_running, "waiting": eng.num_waiting,
                "kv_free_pages": kv["free"] + kv["evictable"], "kv_total_pages": kv["num_blocks"],
                "prefix_hit_tokens": kv["hit_tokens"], "prompt_tokens": kv["query_tokens"],
                "output_tokens": eng.stats["output_tokens"], "steps": eng.stats["steps"],
                "preemptions": eng.sched.num_preemptions, "perf": eng.perf_stats()}

    def shutdown(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=10)


def _put_all(items) -> None:
    for q, o in items:
        q.put_nowait(o)


def _merge(first: StepOutput, q: asyncio.Queue):
    """Fold the outputs already waiting in ``q`` into ``first`` (token ids concatenated, the last one's status): one
    pass through the provider / agent / SSE layers per wakeup instead of one per token when the API loop is busy."""
    ids = list(first.new_token_ids)
    last = first
    while not q.empty():
        o = q.get_nowait()
        if isinstance(o, BaseException):
            return o
        ids += o.new_token_ids
        last = o
        if o.finished:
            break
    return StepOutput(last.request_id, ids, last.finished, last.finish_reason, last.num_prompt_tokens,
                      last.num_output_tokens, last.num_cached_tokens)
