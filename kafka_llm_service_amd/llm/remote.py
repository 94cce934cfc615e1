"""RemoteOpenAIProvider: an LLMProvider for any OpenAI-compatible ``/v1/chat/completions`` endpoint, over httpx.

The reference's only provider was a gateway client (/root/reference/src/llm/portkey.py:62-701: per-request client,
provider routing by model name, tool-call delta normalisation, a default ``max_tokens`` for some vendors). The north
star replaces it with the on-node engine, but deployments still need to chain to another OpenAI-compatible server —
another kafka-llm-service-amd node, a separate model server, or a hosted API — for example as the summariser of the
context-compaction provider. This is that client, without vendor SDKs (``openai`` / ``portkey_ai`` are not
installed here):

* one pooled ``httpx.AsyncClient`` (the reference built a new client per request, portkey.py:341-371),
* request = OpenAI chat-completions JSON (messages via ``Message.to_dict``, tools, sampling knobs, ``stream: true``
  with ``stream_options.include_usage``), auth from ``api_key`` / ``OPENAI_API_KEY``, extra headers pass-through,
* response SSE parsed incrementally; ``content`` deltas, ``tool_calls`` deltas (normalised to
  ``index/id/type/function{name, arguments}``, portkey.py:447-464), ``finish_reason`` and ``usage`` are mapped onto
  ``StreamChunk``s; HTTP errors become ``LLMProviderError`` with the upstream status and message, so context-length
  errors from the remote trigger the agent's compaction path like local ones.
"""
from __future__ import annotations

import json
import os
from typing import Any, AsyncGenerator, Optional

import httpx

from kafka_llm_service_amd.llm.base import LLMProvider
from kafka_llm_service_amd.llm.types import LLMProviderError, Message, StreamChunk, Usage


class RemoteOpenAIProvider(LLMProvider):
    def __init__(self, base_url: str, model: str, api_key: str | None = None, headers: dict | None = None,
                 default_max_tokens: int | None = None, timeout: float = 600.0, tool_provider=None,
                 transport: httpx.AsyncBaseTransport | None = None):
        super().__init__(tool_provider)
        self.base_url = base_url.rstrip("/")
        self.model = model
        self.default_max_tokens = default_max_tokens
        key = api_key or os.environ.get("OPENAI_API_KEY")
        h = {"Content-Type": "application/json", **(headers or {})}
        if key:
            h["Authorization"] = f"Bearer {key}"
        self._client = httpx.AsyncClient(base_url=self.base_url, headers=h, timeout=timeout, transport=transport)

    async def aclose(self) -> None:
        await self._client.aclose()

    def _body(self, messages: list[Message], temperature, max_tokens, stop, tools, kw) -> dict:
        body: dict[str, Any] = {"model": kw.pop("model", None) or self.model,
                                "messages": [m.to_dict() for m in messages], "stream": True,
                                "stream_options": {"include_usage": True}}
        if temperature is not None:
            body["temperature"] = temperature
        mt = max_tokens or self.default_max_tokens
        if mt:
            body["max_tokens"] = mt
        if stop:
            body["stop"] = stop
        if tools:
            body["tools"] = tools
        for k in ("top_p", "frequency_penalty", "presence_penalty", "seed", "user", "tool_choice"):
            if kw.get(k) is not None:
                body[k] = kw[k]
        return body

    async def stream_completion(self, messages: list[Message], *, temperature: Optional[float] = None,
                                max_tokens: Optional[int] = None, stop: Optional[list[str]] = None,
                                tools: Optional[list[dict]] = None, **kwargs: Any) -> AsyncGenerator[StreamChunk, None]:
        self.validate_messages(messages)
        if tools is None:
            tools = await self.get_tools()
        kwargs.pop("routing_key", None)
        body = self._body(messages, temperature, max_tokens, stop, tools, dict(kwargs))
        try:
            async with self._client.stream("POST", "/chat/completions", json=body) as r:
                if r.status_code >= 400:
                    raw = (await r.aread()).decode(errors="replace")
                    try:
                        msg = json.loads(raw).get("error", {}).get("message") or raw
                    except (json.JSONDecodeError, AttributeError):
                        msg = raw
                    raise LLMProviderError(str(msg), provider="remote", status_code=r.status_code)
                buf = ""
                async for piece in r.aiter_text():
                    buf += piece
                    while "\n\n" in buf:
                        frame, buf = buf.split("\n\n", 1)
                        for ch in self._frame(frame):
                            if ch is None:
                                return
                            yield ch
                if buf.strip():
                    for ch in self._frame(buf):
                        if ch is None:
                            return
                        yield ch
        except httpx.HTTPError as e:
            raise LLMProviderError(f"remote provider unreachable: {e}", provider="remote") from e

    def _frame(self, frame: str):
        """One SSE event -> StreamChunks (``None`` marks [DONE])."""
        data = "\n".join(line[5:].lstrip() for line in frame.splitlines() if line.startswith("data:"))
        if not data:
            return []
        if data == "[DONE]":
            return [None]
        d = json.loads(data)
        if "error" in d:
            e = d["error"]
            raise LLMProviderError(e.get("message", str(e)) if isinstance(e, dict) else str(e), provider="remote")
        out = []
        usage = d.get("usage")
        for c in d.get("choices") or []:
            delta = c.get("delta") or {}
            calls = None
            if delta.get("tool_calls"):
                calls = []
                for tc in delta["tool_calls"]:
                    fn = tc.get("function") or {}
                    n = {"index": tc.get("index", 0)}
                    if tc.get("id"):
                        n["id"] = tc["id"]
                        n["type"] = "function"
                    f = {}
                    if fn.get("name"):
                        f["name"] = fn["name"]
                    if fn.get("arguments") is not None:
                        f["arguments"] = fn["arguments"]
                    if f:
                        n["function"] = f
                    calls.append(n)
            if delta.get("role") or delta.get("content") or calls or c.get("finish_reason"):
                out.append(StreamChunk(role=delta.get("role"), content=delta.get("content"), tool_calls=calls,
                                       finish_reason=c.get("finish_reason"), model=d.get("model"), id=d.get("id")))
        if usage:
            out.append(StreamChunk(id=d.get("id"), model=d.get("model"),
                                   usage=Usage(prompt_tokens=usage.get("prompt_tokens", 0),
                                               completion_tokens=usage.get("completion_tokens", 0),
                                               total_tokens=usage.get("total_tokens", 0))))
        return out

    def get_model_info(self) -> dict[str, Any]:
        return {"provider": "remote-openai", "base_url": self.base_url, "model": self.model}
