"""Message / stream-chunk / completion types shared by every LLM provider.

Contract parity with /root/reference/src/llm/types.py:14-184 (Role, Message with ``to_dict`` dropping None fields,
StreamChunk with ``delta`` / ``is_final``, CompletionResponse, LLMProviderError). ``Usage`` is new: the engine
reports real token counts (the reference always returned zeros, quirk Q8).
"""
from __future__ import annotations

from enum import Enum
from typing import Any, Optional

from pydantic import BaseModel, Field


class Role(str, Enum):
    SYSTEM = "system"
    USER = "user"
    ASSISTANT = "assistant"
    TOOL = "tool"


class Message(BaseModel):
    role: str
    content: Optional[str] = None
    name: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None
    tool_call_id: Optional[str] = None
    # engine token cache: the exact token ids the engine generated for this assistant message.
    # Never serialised to clients; lets the chat template reproduce the generated prefix bit-exactly.
    token_ids: Optional[list[int]] = Field(default=None, exclude=True)

    def to_dict(self) -> dict[str, Any]:
        d: dict[str, Any] = {"role": self.role}
        for k in ("content", "name", "tool_calls", "tool_call_id"):
            v = getattr(self, k)
            if v is not None:
                d[k] = v
        return d

    @classmethod
    def from_dict(cls, d: dict[str, Any]) -> "Message":
        content = d.get("content")
        if isinstance(content, list):  # multi-part content -> text (reference: src/db/local.py:123-132)
            content = "\n".join(p.get("text", "") if isinstance(p, dict) else str(p) for p in content)
        return cls(role=d.get("role", "user"), content=content, name=d.get("name"), tool_calls=d.get("tool_calls"),
                   tool_call_id=d.get("tool_call_id"), token_ids=d.get("token_ids"))


class Usage(BaseModel):
    prompt_tokens: int = 0
    completion_tokens: int = 0
    total_tokens: int = 0
    cached_tokens: int = 0


class StreamChunk(BaseModel):
    content: Optional[str] = None
    role: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None
    finish_reason: Optional[str] = None
    model: Optional[str] = None
    id: Optional[str] = None
    usage: Optional[Usage] = None
    token_ids: Optional[list[int]] = None  # engine token ids of this chunk (for the thread token cache)

    @property
    def delta(self) -> str:
        return self.content or ""

    @property
    def is_final(self) -> bool:
        return self.finish_reason is not None


class CompletionResponse(BaseModel):
    content: Optional[str] = None
    role: str = "assistant"
    tool_calls: Optional[list[dict[str, Any]]] = None
    finish_reason: Optional[str] = None
    model: Optional[str] = None
    id: Optional[str] = None
    usage: Optional[Usage] = None
    token_ids: Optional[list[int]] = None

    @property
    def message(self) -> Message:
        return Message(role=self.role, content=self.content, tool_calls=self.tool_calls, token_ids=self.token_ids)

    @property
    def has_tool_calls(self) -> bool:
        return bool(self.tool_calls)


class LLMProviderError(Exception):
    def __init__(self, message: str, provider: str | None = None, status_code: int | None = None,
                 original_error: Exception | None = None):
        super().__init__(message)
        self.message = message
        self.provider = provider
        self.status_code = status_code
        self.original_error = original_error

    def __str__(self) -> str:
        parts = [self.message]
        if self.provider:
            parts.insert(0, f"[{self.provider}]")
        if self.status_code:
            parts.append(f"(status {self.status_code})")
        return " ".join(parts)
