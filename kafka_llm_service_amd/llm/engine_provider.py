"""EngineLLMProvider: the LLMProvider backed by the on-node MI355X engine (replaces the Portkey gateway provider,
/root/reference/src/llm/portkey.py:62-701, per the north star).

Per call: render the chat template (system prompt + tool schemas + history, re-using stored engine token ids) to
token ids -> refuse up front with an OpenAI-style "maximum context length" error if it cannot fit (the agent's
compaction path recognises it, /root/reference/src/llm/context_compaction/base.py:42-43) -> submit to the engine
(routed by thread id for KV affinity) -> detokenize incrementally and yield live content chunks -> a generation that
opens with the tool-call token (``<|python_tag|>`` / ``[TOOL_CALLS]``) is parsed into OpenAI ``tool_calls`` deltas
(``index``/``id``/``type``/``function{name, arguments}``, the normalised shape the Portkey provider produced,
portkey.py:447-464); with tools present the sampler runs the tool-call grammar of ``engine/constrained.py``, so a call
is always well-formed, and ``tool_choice`` ("auto" / "required" / "none" / a named function) is honoured -> a final chunk with ``finish_reason`` and real ``usage``. Every chunk carries the generated
token ids so the agent can store them with the message (thread token cache).
"""
from __future__ import annotations

import asyncio
import os
import time
import uuid
from typing import Any, AsyncGenerator

import numpy as np

from kafka_llm_service_amd.engine.chat_template import ChatTemplate, parse_tool_calls
from kafka_llm_service_amd.engine.sequence import SamplingParams
from kafka_llm_service_amd.engine.tokenizer import IncrementalDetokenizer, tokenizer_for_model
from kafka_llm_service_amd.llm.base import LLMProvider
from kafka_llm_service_amd.llm.types import LLMProviderError, Message, StreamChunk, Usage
from kafka_llm_service_amd.obs import trace


def _gpu_host() -> bool:
    """GPUs visible to this process (counting them does not initialise HIP here: the engine owns the devices)."""
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


class EngineLLMProvider(LLMProvider):
    def __init__(self, client, default_max_tokens: int = 1024, model_name: str = "llama3-8b", tool_provider=None,
                 ignore_eos: bool = False, constrain_tools: bool = True, tool_choice: Any = "auto"):
        super().__init__(tool_provider)
        # schema-constrained tool calls (engine/constrained.py): every call the model opens is well-formed JSON
        # matching the tool's schema; tool_choice "required" / a named function forces one (random-init weights)
        self.constrain_tools = constrain_tools
        self.tool_choice = tool_choice
        self.client = client
        self.tok = tokenizer_for_model(client.model_cfg)
        self.template = ChatTemplate(self.tok)
        self.default_max_tokens = default_max_tokens
        self.model_name = model_name
        self.ignore_eos = ignore_eos
        self._tool_start = self.template.tool_call_start_ids()
        self._pin: list[int] | None = None
        self._pin_key = None

    def _choice(self, tool_choice: Any, messages: list[Message]) -> Any:
        """The request's tool_choice, else the server default; a LIST default is a per-iteration script: entry i for
        the i-th LLM call of the turn (i = assistant tool-call messages after the last user message)."""
        tc = tool_choice or self.tool_choice
        if isinstance(tc, list):
            i = 0
            for m in reversed(messages):
                if m.role == "user":
                    break
                if m.role == "assistant" and m.tool_calls:
                    i += 1
            tc = tc[min(i, len(tc) - 1)] if tc else "auto"
        return tc

    def render(self, messages: list[Message], tools: list[dict] | None) -> list[int]:
        return self.template.render(messages, tools)

    async def warm(self, system_prompt: str, tools: list[dict] | None) -> int:
        """Prefill the shared system prefix (system prompt + tool schemas) on every engine replica and pin it, so the
        very first request of every thread is a prefix hit (SURVEY.md §3.1 target: "pre-fill the shared
        system-prefix KV on each replica ... then start the API"). Returns the prefix length in tokens."""
        ids = self.template.render([Message(role="system", content=system_prompt)], tools,
                                   add_generation_prompt=False)
        if hasattr(self.client, "warm_prefix"):
            await self.client.warm_prefix(ids)
            self._pin = ids
            n = int(os.environ.get("KAFKA_WARM_BURST", "64" if _gpu_host() else "0"))
            if n > 0:
                await self._warm_burst(ids, n)
        return len(ids)

    async def _warm_burst(self, prefix: list[int], n: int) -> None:
        """A burst of ``n`` short requests behind the pinned prefix (tails of 8..103 tokens, 8 sampled tokens each)
        before the API opens: the decode steps of 1..n rows and the mixed steps of the many row counts a burst of new
        turns produces run once, so their kernels are loaded and their GEMM shapes resolved (hipBLASLt heuristics on
        the first call of a shape) before the first real burst instead of inside it."""
        rng = np.random.default_rng(0)
        sp = SamplingParams(temperature=0.7, max_tokens=8, ignore_eos=True, seed=1)
        pre = list(prefix)

        async def one(i: int) -> None:
            tail = [pre[j] for j in rng.integers(0, len(pre), size=8 + (i * 7) % 96)]
            async for _ in self.client.generate(f"warm-burst-{i}", pre + tail, sp, f"warm-burst-{i}"):
                pass
        await asyncio.gather(*(one(i) for i in range(n)))

    def _maybe_pin(self, messages: list[Message], tools: list[dict] | None) -> None:
        """Pin the shared system prefix (system prompt + tool schemas, ~18k tokens for Kafka) in the engine's prefix
        cache once it has been computed, so KV pressure from long threads never evicts it. With per-thread prompt
        tails (profiles, playbooks) only the common part of all system prefixes seen so far stays pinned."""
        if not messages or messages[0].role != "system" or not hasattr(self.client, "pin_prefix"):
            return
        # fast path (every request of a thread with the same system prompt + tool set): no render, no compare —
        # this runs on the API event loop once per request (it cost ~0.65 ms per request before)
        key = (hash(messages[0].content or ""), tuple((t.get("function") or {}).get("name", "") for t in tools or ()))
        if key == self._pin_key:
            return
        self._pin_key = key
        ids = self.template.render(messages[:1], tools)
        if self._pin is not None:
            m = min(len(self._pin), len(ids))
            a, b = np.asarray(self._pin[:m]), np.asarray(ids[:m])
            diff = np.flatnonzero(a != b)
            n = int(diff[0]) if diff.size else m
            if n == len(self._pin):
                return
            ids = ids[:n]
        if len(ids) < 256:  # nothing worth pinning in common
            self._pin = ids
            return
        self._pin = ids
        self.client.pin_prefix(ids)

    async def stream_completion(self, messages: list[Message], *, temperature: float | None = None,
                                max_tokens: int | None = None, stop: list[str] | None = None,
                                tools: list[dict] | None = None, top_p: float | None = None,
                                frequency_penalty: float | None = None, presence_penalty: float | None = None,
                                seed: int | None = None, routing_key: str | None = None,
                                tool_choice: Any = None, **kwargs: Any) -> AsyncGenerator[StreamChunk, None]:
        self.validate_messages(messages)
        if tools is None:
            tools = await self.get_tools()
        with trace.span("api_render", "api", f"thr:{routing_key}", messages=len(messages)):
            prompt = self.render(messages, tools)
        limit = self.client.max_model_len
        if len(prompt) + 1 > limit:
            raise LLMProviderError(f"This model's maximum context length is {limit} tokens. However, your messages "
                                   f"resulted in {len(prompt)} tokens.", provider="engine", status_code=400)
        max_new = min(max_tokens or self.default_max_tokens, limit - len(prompt))
        params = SamplingParams(temperature=0.7 if temperature is None else float(temperature),
                                top_p=1.0 if not top_p else float(top_p), max_tokens=max_new,
                                frequency_penalty=float(frequency_penalty or 0.0),
                                presence_penalty=float(presence_penalty or 0.0), seed=seed,
                                ignore_eos=self.ignore_eos,
                                tool_grammar=({"tools": tools, "tool_choice": self._choice(tool_choice, messages)}
                                              if tools and self.constrain_tools else None))
        stops = [s for s in (stop or []) if s]
        hold = max((len(s) for s in stops), default=1) - 1
        rid = f"req-{uuid.uuid4().hex}"
        cid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        yield StreamChunk(role="assistant", id=cid, model=self.model_name)
        detok = IncrementalDetokenizer(self.tok)
        mode = None
        tool_ids: list[int] = []
        all_ids: list[int] = []
        pending = ""
        finish = "stop"
        cached = 0
        n_out = 0
        stopped = False
        tr = trace.tracer()
        t_sub = time.perf_counter()
        async for out in self.client.generate(rid, prompt, params, routing_key):
            ids = out.new_token_ids
            if tr is not None and n_out == 0:  # submit -> first engine output on this (API) loop
                tr.complete("api_engine_first", "api", t_sub, time.perf_counter(), f"thr:{routing_key}",
                            {"prompt_tokens": len(prompt), "cached": out.num_cached_tokens})
            all_ids.extend(ids)
            n_out = out.num_output_tokens
            cached = out.num_cached_tokens
            if mode is None and ids:
                mode = "tool" if ids[0] in self._tool_start else "text"
            if mode == "tool":
                tool_ids.extend(i for i in ids if not self.tok.is_special(i))
            else:
                text = detok.add(ids)
                if text:
                    pending += text
                    if stops:
                        cut = min((pending.find(s) for s in stops if s in pending), default=-1)
                        if cut >= 0:
                            if pending[:cut]:
                                yield StreamChunk(content=pending[:cut], id=cid)
                            finish, stopped = "stop", True
                            break
                    emit = pending[:len(pending) - hold] if hold else pending
                    if emit:
                        pending = pending[len(emit):]
                        yield StreamChunk(content=emit, id=cid)
            if out.finished:
                finish = out.finish_reason or "stop"
        if mode != "tool" and pending and not stopped:
            yield StreamChunk(content=pending, id=cid)
        calls = None
        if mode == "tool":
            body = self.tok.decode(tool_ids)
            calls = parse_tool_calls(body)
            if calls is None:  # malformed call: surface the raw text instead of inventing arguments
                yield StreamChunk(content=body, id=cid)
            else:
                for c in calls:
                    yield StreamChunk(tool_calls=[{"index": c["index"], "id": c["id"], "type": "function",
                                                   "function": {"name": c["function"]["name"], "arguments": ""}}],
                                      id=cid)
                    yield StreamChunk(tool_calls=[{"index": c["index"],
                                                   "function": {"arguments": c["function"]["arguments"]}}], id=cid)
        if finish == "abort":
            finish = "stop"
        self._maybe_pin(messages, tools)
        yield StreamChunk(finish_reason="tool_calls" if calls else finish, id=cid, token_ids=all_ids,
                          usage=Usage(prompt_tokens=len(prompt), completion_tokens=n_out,
                                      total_tokens=len(prompt) + n_out, cached_tokens=cached))
