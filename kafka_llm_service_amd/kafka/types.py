"""OpenAI-compatible request / response schemas (/root/reference/src/kafka/types.py:13-107).

Same field names and validation bounds (temperature in [0, 2], max_tokens > 0, top_p in [0, 1], penalties in
[-2, 2]). ``usage`` is populated from real engine token counts (quirk Q8); ``stream_options.include_usage`` adds a
final usage chunk like the OpenAI API; ``tool_choice`` / ``tools`` are accepted (the server's own tool set is used,
``tool_choice`` steers constrained decoding).
"""
from __future__ import annotations

from typing import Any, Optional

from pydantic import BaseModel, Field


class ChatMessage(BaseModel):
    role: str
    content: Optional[str] = None
    name: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None
    tool_call_id: Optional[str] = None


class StreamOptions(BaseModel):
    include_usage: bool = False


class ChatCompletionRequest(BaseModel):
    model: str
    messages: list[ChatMessage]
    temperature: Optional[float] = Field(None, ge=0, le=2)
    max_tokens: Optional[int] = Field(None, gt=0)
    stream: Optional[bool] = False
    stop: Optional[list[str] | str] = None
    top_p: Optional[float] = Field(None, ge=0, le=1)
    frequency_penalty: Optional[float] = Field(None, ge=-2, le=2)
    presence_penalty: Optional[float] = Field(None, ge=-2, le=2)
    user: Optional[str] = None
    seed: Optional[int] = None
    stream_options: Optional[StreamOptions] = None
    tool_choice: Optional[Any] = None
    tools: Optional[list[dict[str, Any]]] = None


class AgentRunRequest(BaseModel):
    messages: list[ChatMessage]
    model: str = "default"
    temperature: float = 0.7
    max_tokens: Optional[int] = None


class CreateThreadRequest(BaseModel):
    system_message: Optional[str] = None
    user_id: Optional[str] = None
    kafka_profile_id: Optional[str] = None
    metadata: Optional[dict[str, Any]] = None


class DeltaContent(BaseModel):
    role: Optional[str] = None
    content: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None


class StreamChoice(BaseModel):
    index: int = 0
    delta: DeltaContent
    finish_reason: Optional[str] = None


class StreamChunkResponse(BaseModel):
    id: str
    object: str = "chat.completion.chunk"
    created: int
    model: str
    choices: list[StreamChoice]


class MessageContent(BaseModel):
    role: str = "assistant"
    content: Optional[str] = None
    tool_calls: Optional[list[dict[str, Any]]] = None


class Choice(BaseModel):
    index: int = 0
    message: MessageContent
    finish_reason: Optional[str] = None


class Usage(BaseModel):
    prompt_tokens: int = 0
    completion_tokens: int = 0
    total_tokens: int = 0


class ChatCompletionResponse(BaseModel):
    id: str
    object: str = "chat.completion"
    created: int
    model: str
    choices: list[Choice]
    usage: Optional[Usage] = None
