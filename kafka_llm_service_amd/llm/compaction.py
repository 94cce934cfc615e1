"""Context compaction: what the agent does when a completion is refused for exceeding the context window.

Parity with /root/reference/src/llm/context_compaction/base.py:10-221 and v1.py:20-313:
  * ``is_context_length_error`` recognises every provider phrasing the reference recognises — and the engine raises
    ``"This model's maximum context length is N tokens..."`` BEFORE any GPU work (engine/engine.py add_request),
  * ``find_safe_split_point`` never separates an assistant tool-call message from its tool results,
  * ``validate_message_structure`` drops orphan tool results and empty assistant messages,
  * ``SummarizationCompactionProvider`` summarises the oldest ~75% (min 10 messages) with the LLM at T=0.3 and keeps
    the newest ~25% verbatim; ``TruncationCompactionProvider`` keeps the last N.
Fixed vs the reference (quirk Q5): the summary is a plain-string system message (the reference built list content,
which its ``Message`` type rejects, so its summariser always failed) and the summariser is any ``LLMProvider``
(here: the on-node engine) instead of a raw OpenAI client.
"""
from __future__ import annotations

import json
import logging
from abc import ABC, abstractmethod
from typing import Any

_PATTERNS_ALL = [
    ("prompt is too long", "tokens"), ("input is too long",), ("input length and", "max_tokens", "exceed context limit"),
    ("context_length_exceeded",), ("maximum context length",), ("token limit",), ("exceeds the maximum", "token"),
    ("too many tokens",), ("exceeds maximum", "tokens"),
]

MODEL_MAX_OUTPUT_TOKENS = {"gpt-4o": 16384, "gpt-4o-mini": 16384, "gpt-5": 32768, "claude-sonnet-4-5": 16384,
                           "claude-3-5-sonnet": 8192, "claude-3-opus": 4096, "gemini-2.0-flash": 8192,
                           "gemini-2.5-pro": 65536, "gemini-2.5-flash": 65536, "llama3": 8192, "mixtral": 8192}

SUMMARY_PROMPT = (
    "You write the hand-off summary of a long conversation so that it can continue in a fresh context.\n"
    "Keep: every decision and action taken, facts and data discovered, tool calls and their outcomes, errors, "
    "the user's stated requirements and preferences, and the exact state of unfinished work.\n"
    "Write markdown with short sections: Goal, Progress, Findings, Open items.")


def is_context_length_error(error: Exception) -> bool:
    texts = [str(error).lower()]
    body = getattr(error, "body", None)
    if body:
        texts.append(str(body).lower())
    for t in texts:
        for pat in _PATTERNS_ALL:
            if all(p in t for p in pat):
                return True
    return False


def get_max_output_tokens(model: str) -> int:
    if model in MODEL_MAX_OUTPUT_TOKENS:
        return MODEL_MAX_OUTPUT_TOKENS[model]
    for k, v in MODEL_MAX_OUTPUT_TOKENS.items():
        if model.startswith(k):
            return v
    return 8192


def find_safe_split_point(messages: list[dict[str, Any]], target: int) -> int:
    if target <= 0:
        return 0
    if target >= len(messages):
        return len(messages)
    i = target
    while i > 0:
        prev, nxt = messages[i - 1], messages[i] if i < len(messages) else None
        if prev.get("role") == "assistant" and prev.get("tool_calls"):
            i -= 1
            continue
        if nxt is not None and nxt.get("role") == "tool":
            i -= 1
            continue
        break
    return i


def validate_message_structure(messages: list[dict[str, Any]], logger: logging.Logger | None = None):
    ids = {tc.get("id") for m in messages if m.get("role") == "assistant" and m.get("tool_calls")
           for tc in m["tool_calls"] if tc.get("id")}
    out = []
    for m in messages:
        if m.get("role") == "tool" and m.get("tool_call_id") not in ids:
            if logger:
                logger.warning("dropping orphan tool result %s", m.get("tool_call_id"))
            continue
        if m.get("role") == "assistant" and not m.get("content") and not m.get("tool_calls"):
            if logger:
                logger.warning("dropping empty assistant message")
            continue
        out.append(m)
    return out


def _split_system_head(messages):
    head, rest = [], []
    for m in messages:
        if m.get("role") == "system" and not rest:
            head.append(m)
        else:
            rest.append(m)
    return head, rest


class ContextCompactionProvider(ABC):
    def __init__(self, logger: logging.Logger | None = None):
        self.logger = logger or logging.getLogger("kafka.compaction")

    @abstractmethod
    async def compact(self, messages: list[dict[str, Any]], system_prompt: str, model: str,
                      **kwargs: Any) -> list[dict[str, Any]]:
        ...

    def should_compact(self, error: Exception) -> bool:
        return is_context_length_error(error)


class TruncationCompactionProvider(ContextCompactionProvider):
    def __init__(self, keep_last: int = 50, logger: logging.Logger | None = None):
        super().__init__(logger)
        self.keep_last = keep_last

    async def compact(self, messages, system_prompt, model, **kwargs):
        head, rest = _split_system_head(messages)
        if len(rest) <= self.keep_last:
            return messages
        start = len(rest) - self.keep_last
        # move the cut forward past any tool results whose call would be cut off
        while start < len(rest) and rest[start].get("role") == "tool":
            start += 1
        return validate_message_structure(head + rest[start:], self.logger)


class SummarizationCompactionProvider(ContextCompactionProvider):
    def __init__(self, llm_provider, summarize_ratio: float = 0.75, min_messages_to_summarize: int = 10,
                 fallback: ContextCompactionProvider | None = None, logger: logging.Logger | None = None):
        super().__init__(logger)
        self.llm = llm_provider
        self.summarize_ratio = summarize_ratio
        self.min_messages = min_messages_to_summarize
        self.fallback = fallback or TruncationCompactionProvider(logger=logger)

    async def compact(self, messages, system_prompt, model, **kwargs):
        from kafka_llm_service_amd.llm.types import Message

        head, rest = _split_system_head(messages)
        if len(rest) < self.min_messages:
            return messages
        split = find_safe_split_point(rest, int(len(rest) * self.summarize_ratio))
        old, keep = rest[:split], rest[split:]
        if not old:
            return messages
        req = [Message(role="system", content=SUMMARY_PROMPT),
               Message(role="user", content="Summarize this conversation history:\n\n" + json.dumps(old, indent=1))]
        try:
            resp = await self.llm.completion(req, temperature=0.3,
                                             max_tokens=min(8192, get_max_output_tokens(model) // 4), model=model)
            summary = resp.content or ""
        except Exception as e:  # summariser failed: fall back to truncation instead of giving up
            self.logger.warning("summarization failed (%s); truncating", e)
            return await self.fallback.compact(messages, system_prompt, model)
        note = {"role": "system",
                "content": f"[CONVERSATION HANDOFF - {len(old)} messages summarized]\n\n{summary}"}
        return validate_message_structure(head + [note] + keep, self.logger)
