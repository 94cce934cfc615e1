"""The agent loop: LLM -> tool calls -> tool results -> LLM ... until the model stops calling tools or calls ``idle``.

Event grammar parity with /root/reference/src/agents/base.py:160-440 (the golden traces of SURVEY.md §2.5.2):
  * OpenAI ``chat.completion.chunk`` dicts (only present delta keys; a new chunk id per LLM iteration),
  * ``{"type": "tool_result", "tool_call_id", "tool_name", "delta", "is_complete"}`` while tools run (tools execute
    sequentially; an ``idle`` call ends the run immediately, quirk Q13; bad argument JSON becomes ``{}``, Q14),
  * ``{"type": "agent_done", "reason": "text_response" | "idle" | "max_iterations", ...}``.
Changed on purpose (quirk Q2): chunks are yielded LIVE as the engine produces tokens — the reference buffered every
LLM turn before emitting anything, so its time-to-first-token was the whole turn. Context-length errors are raised by
the engine before the first token, which is when compaction is still possible; the loop retries once after
compaction, as the reference does. The engine's token ids of each assistant turn are kept on the message
(``Message.token_ids``) so the next iteration re-renders it bit-exactly and hits the prefix cache.
"""
from __future__ import annotations

import json
import logging
import time
import uuid
from typing import Any, AsyncGenerator

from kafka_llm_service_amd.llm.base import accumulate_tool_calls
from kafka_llm_service_amd.llm.compaction import is_context_length_error
from kafka_llm_service_amd.llm.types import Message
from kafka_llm_service_amd.tools.types import Tool


def _tool_done(name: str, t0: float) -> None:
    """Tool time (SURVEY.md §5.1 spans / §5.5 metrics)."""
    from kafka_llm_service_amd.obs import metrics, trace

    t1 = time.perf_counter()
    metrics.TOOL_SECONDS.labels(tool=name).observe(t1 - t0)
    tr = trace.tracer()
    if tr is not None:
        tr.complete(f"tool:{name}", "agent", t0, t1)

IDLE_TOOL_NAME = "idle"


def make_idle_tool() -> Tool:
    return Tool(
        name=IDLE_TOOL_NAME,
        description="Call this after using tools to signal you are done with your task. Only needed after tool "
                    "usage, not for simple text responses.",
        parameters={"type": "object", "properties": {"summary": {
            "type": "string", "description": "Optional brief summary of what was accomplished"}}, "required": []},
        handler=lambda summary="": {"status": "idle", "summary": summary})


def message_to_dict(m: Message) -> dict[str, Any]:
    d: dict[str, Any] = {"role": m.role}
    if m.content is not None:
        d["content"] = m.content
    if m.tool_calls:
        d["tool_calls"] = m.tool_calls
    if m.tool_call_id:
        d["tool_call_id"] = m.tool_call_id
    if m.name:
        d["name"] = m.name
    return d


class Agent:
    def __init__(self, llm_provider, tool_provider, system_prompt: str | None = None, prompt_provider=None,
                 context_compaction_provider=None, max_iterations: int = 50, logger: logging.Logger | None = None):
        self.llm_provider = llm_provider
        self.tool_provider = tool_provider
        self.prompt_provider = prompt_provider
        self.context_compaction_provider = context_compaction_provider
        self.max_iterations = max_iterations
        self.logger = logger or logging.getLogger("kafka.agent")
        if system_prompt is not None:
            self.system_prompt = system_prompt
        elif prompt_provider is not None:
            self.system_prompt = prompt_provider.get_system_prompt()
        else:
            self.system_prompt = None
        if not tool_provider.has_tool(IDLE_TOOL_NAME):
            tool_provider.add_tool(make_idle_tool())

    async def run(self, messages: list[Message], model: str = "default", temperature: float = 0.7,
                  max_tokens: int | None = None, emit_messages: bool = False,
                  **kwargs) -> AsyncGenerator[dict[str, Any], None]:
        """Yield agent events. With ``emit_messages`` it also yields ``{"type": "_message", "message": Message}`` for
        every assistant / tool message it appends (with the engine token ids) — consumed by KafkaAgent for
        persistence and never forwarded to clients."""
        working = list(messages)
        if self.system_prompt and (not working or working[0].role != "system"):
            working.insert(0, Message(role="system", content=self.system_prompt))
        tools = await self.tool_provider.get_tools()
        compacted = False
        iteration = 0
        total = {"prompt_tokens": 0, "completion_tokens": 0, "total_tokens": 0, "cached_tokens": 0}
        seen_usage = False

        def done_event(ev: dict) -> dict:
            if seen_usage:
                ev["usage"] = dict(total)
            return ev
        while iteration < self.max_iterations:
            cid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
            created = int(time.time())
            content = ""
            acc: dict[int, dict] = {}
            token_ids: list[int] = []
            usage = None
            stream = self.llm_provider.stream_completion(working, model=model, temperature=temperature,
                                                         max_tokens=max_tokens, tools=tools, **kwargs)
            first = True
            try:
                async for ch in stream:
                    first = False
                    delta: dict[str, Any] = {}
                    if ch.role:
                        delta["role"] = ch.role
                    if ch.content:
                        delta["content"] = ch.content
                        content += ch.content
                    if ch.tool_calls:
                        accumulate_tool_calls(acc, ch.tool_calls)
                        out = []
                        for tc in ch.tool_calls:
                            d: dict[str, Any] = {"index": tc.get("index", 0)}
                            if tc.get("id"):
                                d["id"] = tc["id"]
                                d["type"] = "function"
                            fn = tc.get("function") or {}
                            if fn:
                                d["function"] = {k: fn[k] for k in ("name", "arguments") if fn.get(k)}
                            out.append(d)
                        delta["tool_calls"] = out
                    if ch.token_ids:
                        token_ids.extend(ch.token_ids)
                    if ch.usage:
                        usage = ch.usage
                    yield {"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                           "choices": [{"index": 0, "delta": delta, "finish_reason": ch.finish_reason or None}]}
            except Exception as e:
                if first and not compacted and is_context_length_error(e) and self.context_compaction_provider:
                    self.logger.info("context length exceeded (%s); compacting", e)
                    try:
                        new = await self.context_compaction_provider.compact(
                            [message_to_dict(m) for m in working], self.system_prompt or "", model)
                    except Exception as ce:
                        self.logger.error("compaction failed: %s", ce)
                        raise e
                    working = [Message.from_dict(m) for m in new]
                    compacted = True
                    iteration += 1  # the retry consumes an iteration, as in the reference
                    continue
                raise
            if usage is not None:
                seen_usage = True
                for k in total:
                    total[k] += getattr(usage, k, 0) or 0
                # this LLM call's usage as a typed agent event (like tool_result: no ``choices``, so clients that
                # index choices[0] of every chat.completion.chunk keep working): per-iteration prompt / cached tokens
                # show each agent iteration re-using the previous one's KV
                yield {"type": "usage", "id": cid, "iteration": iteration,
                       "usage": {k: getattr(usage, k, 0) or 0 for k in total}}
            calls = [acc[i] for i in sorted(acc)]
            if not calls:
                if emit_messages and content:
                    yield {"type": "_message", "message": Message(role="assistant", content=content,
                                                                  token_ids=token_ids or None)}
                yield done_event({"type": "agent_done", "reason": "text_response", "final_content": content,
                                  "iteration": iteration})
                return
            working.append(Message(role="assistant", content=content or None, tool_calls=calls,
                                   token_ids=token_ids or None))
            if emit_messages:
                yield {"type": "_message", "message": working[-1]}
            for call in calls:
                name = call["function"]["name"]
                try:
                    args = json.loads(call["function"]["arguments"]) if call["function"]["arguments"] else {}
                except json.JSONDecodeError:
                    args = {}
                if not isinstance(args, dict):
                    args = {}
                if name == IDLE_TOOL_NAME:
                    summary = args.get("summary", "")
                    payload = json.dumps({"status": "idle", "summary": summary})
                    working.append(Message(role="tool", content=payload, tool_call_id=call["id"], name=name))
                    if emit_messages:
                        yield {"type": "_message", "message": working[-1]}
                    yield {"type": "tool_result", "tool_call_id": call["id"], "tool_name": name, "delta": payload,
                           "is_complete": True}
                    yield done_event({"type": "agent_done", "reason": "idle", "summary": summary,
                                      "iteration": iteration})
                    return
                result = ""
                t_tool = time.perf_counter()
                async for chunk in self.tool_provider.run_tool_stream(name, args, call["id"]):
                    result += chunk.delta
                    yield {"type": "tool_result", "tool_call_id": call["id"], "tool_name": name,
                           "delta": chunk.delta, "is_complete": chunk.is_complete}
                _tool_done(name, t_tool)
                working.append(Message(role="tool", content=result, tool_call_id=call["id"], name=name))
                if emit_messages:
                    yield {"type": "_message", "message": working[-1]}
            iteration += 1
        yield done_event({"type": "agent_done", "reason": "max_iterations", "iteration": self.max_iterations})
