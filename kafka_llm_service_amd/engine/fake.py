"""A timing-only stand-in for LLMEngine: the API / pipe / SSE path under serving load without a GPU.

``KAFKA_FAKE_ENGINE_STEP_MS=<ms>`` makes the engine worker process (``engine/client.py``) run this instead of the
model: every ``step()`` takes the given wall time (a decode step of the measured MI355X engine, ~8.5-9 ms for
Llama-3-8B at 64 threads), new requests join the next step as a prefill that costs ``KAFKA_FAKE_PREFILL_US_PER_TOKEN``
extra per uncached prompt token, and every running request gets one token per step (ids drawn from a fixed list of
ordinary word tokens, so detokenization does real work). The serve benchmark then measures the HTTP front end — the
event-loop cost per streamed token, request parsing, history persistence — on the CPU, which is where the HTTP burst
TTFT gap of VERDICT r02 (API vs engine first token) lives. Interface: the subset of LLMEngine that ``serve_pipe``
uses.
"""
from __future__ import annotations

import os
import time
from collections import deque

from kafka_llm_service_amd.engine.sequence import SamplingParams, StepOutput


class FakeEngine:
    def __init__(self, step_ms: float, prefill_us_per_token: float = 2.0, prefix_tokens: int = 0):
        self.step_s = step_ms / 1e3
        self.prefill_s = prefill_us_per_token / 1e6
        self.prefix_tokens = prefix_tokens  # treated as cached (the pinned shared system prefix)
        self.waiting: deque = deque()
        self.running: dict[str, list] = {}  # rid -> [n_prompt, n_out, max_tokens]
        self.stats = {"steps": 0, "output_tokens": 0}
        self._next = time.perf_counter()
        self._vocab = [1000 + 7 * i for i in range(512)]

    def add_request(self, request_id: str, prompt_ids: list[int], params: SamplingParams | None = None, meta=None):
        p = params or SamplingParams()
        self.waiting.append((request_id, len(prompt_ids), max(1, p.max_tokens)))

    def abort(self, request_id: str) -> None:
        self.running.pop(request_id, None)
        self.waiting = deque(w for w in self.waiting if w[0] != request_id)

    def has_unfinished(self) -> bool:
        return bool(self.waiting or self.running)

    @property
    def num_running(self) -> int:
        return len(self.running)

    @property
    def num_waiting(self) -> int:
        return len(self.waiting)

    def pin_prefix(self, token_ids: list[int]) -> int:
        self.prefix_tokens = max(self.prefix_tokens, len(token_ids))
        return len(token_ids)

    def kv_stats(self) -> dict:
        return {"num_blocks": 1 << 16, "free": 1 << 16, "evictable": 0, "hit_tokens": 0}

    def perf_stats(self) -> dict:
        """The health message's perf block (LLMEngine.perf_stats): no GPU, only the step count."""
        return {"device": "fake", "steps": self.stats["steps"]}

    def step(self) -> list[StepOutput]:
        cost = self.step_s
        while self.waiting:
            rid, n_prompt, max_tokens = self.waiting.popleft()
            cost += max(0, n_prompt - self.prefix_tokens) * self.prefill_s
            self.running[rid] = [n_prompt, 0, max_tokens]
        self._next = max(self._next + cost, time.perf_counter())
        while True:  # the step's wall time (sleep, then spin the last few hundred microseconds)
            left = self._next - time.perf_counter()
            if left <= 0:
                break
            time.sleep(left - 3e-4) if left > 5e-4 else None
        outs = []
        for rid, st in list(self.running.items()):
            st[1] += 1
            fin = st[1] >= st[2]
            outs.append(StepOutput(rid, [self._vocab[(st[1] * 31 + len(rid)) % len(self._vocab)]], fin,
                                   "length" if fin else None, st[0], st[1], self.prefix_tokens))
            if fin:
                del self.running[rid]
        self.stats["steps"] += 1
        self.stats["output_tokens"] += len(outs)
        return outs


def from_env() -> FakeEngine | None:
    ms = os.environ.get("KAFKA_FAKE_ENGINE_STEP_MS")
    if not ms:
        return None
    return FakeEngine(float(ms), float(os.environ.get("KAFKA_FAKE_PREFILL_US_PER_TOKEN", "2.0")))
