"""LLMProvider: the streaming-first provider interface the agent loop talks to.

Interface parity with /root/reference/src/llm/base.py:67-312 (tool-provider hook, ``get_tools``,
``stream_completion`` / ``completion``, ``validate_messages``, ``get_model_info``). ``completion`` has a default
implementation that folds ``stream_completion`` (tool-call deltas accumulated by ``index`` exactly like the agent
loop does), so a provider only has to implement streaming. Implementations here:
  * ``EngineLLMProvider`` (llm/engine_provider.py) — the on-node MI355X engine (replaces the Portkey provider),
  * ``RemoteOpenAIProvider`` (llm/remote.py) — any OpenAI-compatible HTTP endpoint (the gateway role of the
    reference's Portkey provider, without vendor SDKs),
  * ``StubEchoProvider`` / ``ScriptedProvider`` (llm/stub.py) — BASELINE config 1 and tests.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, AsyncGenerator, Optional

from kafka_llm_service_amd.llm.types import CompletionResponse, Message, StreamChunk, Usage

VALID_ROLES = {"system", "user", "assistant", "tool"}


def accumulate_tool_calls(acc: dict[int, dict], deltas: list[dict]) -> None:
    """Merge OpenAI streaming tool-call deltas (keyed by ``index``) into ``acc``."""
    for tc in deltas:
        idx = tc.get("index", 0)
        fn = tc.get("function") or {}
        cur = acc.setdefault(idx, {"id": tc.get("id", ""), "type": "function",
                                   "function": {"name": fn.get("name", ""), "arguments": ""}})
        if fn.get("arguments"):
            cur["function"]["arguments"] += fn["arguments"]
        if tc.get("id"):
            cur["id"] = tc["id"]
        if fn.get("name"):
            cur["function"]["name"] = fn["name"]


class LLMProvider(ABC):
    def __init__(self, tool_provider=None):
        self._tool_provider = tool_provider

    @property
    def tool_provider(self):
        return self._tool_provider

    @tool_provider.setter
    def tool_provider(self, provider) -> None:
        self._tool_provider = provider

    def has_tools(self) -> bool:
        return self._tool_provider is not None

    async def get_tools(self) -> list[dict[str, Any]]:
        if self._tool_provider is None:
            return []
        return await self._tool_provider.get_tools()

    @abstractmethod
    def stream_completion(self, messages: list[Message], *, temperature: Optional[float] = None,
                          max_tokens: Optional[int] = None, stop: Optional[list[str]] = None,
                          **kwargs: Any) -> AsyncGenerator[StreamChunk, None]:
        """Yield StreamChunks; the last one carries ``finish_reason`` (and ``usage`` when known)."""

    async def completion(self, messages: list[Message], *, temperature: Optional[float] = None,
                         max_tokens: Optional[int] = None, stop: Optional[list[str]] = None,
                         **kwargs: Any) -> CompletionResponse:
        content, finish, model, cid, usage = "", None, None, None, None
        acc: dict[int, dict] = {}
        toks: list[int] = []
        async for ch in self.stream_completion(messages, temperature=temperature, max_tokens=max_tokens, stop=stop,
                                               **kwargs):
            content += ch.delta
            if ch.tool_calls:
                accumulate_tool_calls(acc, ch.tool_calls)
            finish = ch.finish_reason or finish
            model = ch.model or model
            cid = ch.id or cid
            usage = ch.usage or usage
            if ch.token_ids:
                toks.extend(ch.token_ids)
        calls = [acc[i] for i in sorted(acc)] or None
        return CompletionResponse(content=content or None, tool_calls=calls, finish_reason=finish, model=model,
                                  id=cid, usage=usage or Usage(), token_ids=toks or None)

    def validate_messages(self, messages: list[Message]) -> None:
        if not messages:
            raise ValueError("Messages list cannot be empty")
        for i, m in enumerate(messages):
            if m.role not in VALID_ROLES:
                raise ValueError(f"Message {i} has invalid role {m.role!r}")
            if m.role == "tool" and not m.tool_call_id:
                raise ValueError(f"Tool message {i} must have tool_call_id")

    def get_model_info(self) -> dict[str, Any]:
        return {"provider": self.__class__.__name__, "supports_streaming": True, "supports_tools": True}
