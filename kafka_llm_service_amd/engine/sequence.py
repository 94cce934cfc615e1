"""Request / sequence state and sampling parameters of the engine.

``SamplingParams`` carries every OpenAI request knob the reference accepted but dropped on the floor
(/root/reference/src/kafka/types.py:34-38 vs /root/reference/server.py:289-294 — quirk Q7): temperature (0 means
greedy; the reference's ``temperature or 0.7`` coercion, /root/reference/server.py:292, is NOT reproduced — Q6),
top_p, stop, presence/frequency penalties, plus engine-only knobs (top_k, seed, ignore_eos for benchmarks, a logits
processor for constrained tool-call decoding).
"""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Callable


PENDING = -1  # placeholder of a token still being sampled by the in-flight engine step (async scheduling)


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    max_tokens: int = 256
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    # called with (output_token_ids) -> allowed token ids (list / constrained.Mask) or None for "no constraint"
    allowed_tokens_fn: Callable | None = None
    # picklable tool-call grammar {"tools": [...], "tool_choice": ...}: the engine builds the constraint
    # (engine/constrained.py) on its own side, so it also works through the DP / TP worker pipes
    tool_grammar: dict | None = None

    def __post_init__(self):
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0 < self.top_p <= 1:
            raise ValueError("top_p must be in (0, 1]")
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if isinstance(self.stop, str):
            self.stop = [self.stop]

    @property
    def greedy(self) -> bool:
        return self.temperature == 0.0


class SeqStatus(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


_ids = itertools.count(1)


class Sequence:
    __slots__ = ("seq_id", "request_id", "prompt_ids", "output_ids", "params", "status", "num_computed",
                 "num_cached", "arrival", "first_token_time", "finish_reason", "last_token_time", "preemptions",
                 "stop_checker", "meta", "token_times")

    def __init__(self, request_id: str, prompt_ids: list[int], params: SamplingParams, meta: dict | None = None):
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        self.seq_id = next(_ids)
        self.request_id = request_id
        self.prompt_ids = list(prompt_ids)
        self.output_ids: list[int] = []
        self.params = params
        self.status = SeqStatus.WAITING
        self.num_computed = 0
        self.num_cached = 0
        self.arrival = time.perf_counter()
        self.first_token_time: float | None = None
        self.last_token_time: float | None = None
        self.finish_reason: str | None = None
        self.preemptions = 0
        self.stop_checker = None
        self.meta = meta or {}
        self.token_times = None

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    def token_at(self, i: int) -> int:
        n = len(self.prompt_ids)
        return self.prompt_ids[i] if i < n else self.output_ids[i - n]

    def tokens_range(self, a: int, b: int) -> list[int]:
        n = len(self.prompt_ids)
        if b <= n:
            return self.prompt_ids[a:b]
        if a >= n:
            return self.output_ids[a - n:b - n]
        return self.prompt_ids[a:] + self.output_ids[:b - n]

    def all_ids(self) -> list[int]:
        return self.prompt_ids + self.output_ids

    @property
    def remaining(self) -> int:
        return self.total_len - self.num_computed

    @property
    def finished(self) -> bool:
        return self.status == SeqStatus.FINISHED


@dataclass
class StepOutput:
    request_id: str
    new_token_ids: list[int]
    finished: bool
    finish_reason: str | None = None
    num_prompt_tokens: int = 0
    num_output_tokens: int = 0
    num_cached_tokens: int = 0
    text: str | None = None
