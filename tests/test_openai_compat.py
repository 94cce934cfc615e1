"""OpenAI-SDK compatibility of the streaming contract (SURVEY.md §4.4 "Contract": the openai package is not
installable here, so this vendors the parts of openai-python's streaming behaviour a client relies on): every SSE
event of /v1/chat/completions and /v1/threads/{id}/chat/completions validates against ChatCompletionChunk-shaped
models, `chunk.choices[0].delta.content` is safe on every chunk that has choices, the usage chunk has
`choices == []`, and the stream ends with [DONE]."""
import json
from typing import List, Literal, Optional

import pytest
from fastapi.testclient import TestClient
from pydantic import BaseModel, ConfigDict

from kafka_llm_service_amd.db.local import MemoryDBClient
from kafka_llm_service_amd.llm.stub import ScriptedProvider
from kafka_llm_service_amd.server.app import create_app
from kafka_llm_service_amd.server.state import ServerConfig, ServerState


class _M(BaseModel):
    model_config = ConfigDict(extra="allow")


class FunctionDelta(_M):
    name: Optional[str] = None
    arguments: Optional[str] = None


class ToolCallDelta(_M):
    index: int
    id: Optional[str] = None
    type: Optional[Literal["function"]] = None
    function: Optional[FunctionDelta] = None


class Delta(_M):
    role: Optional[Literal["assistant", "user", "system", "tool"]] = None
    content: Optional[str] = None
    tool_calls: Optional[List[ToolCallDelta]] = None


class Choice(_M):
    index: int
    delta: Delta
    finish_reason: Optional[Literal["stop", "length", "tool_calls", "content_filter", "function_call"]] = None


class Usage(_M):
    prompt_tokens: int
    completion_tokens: int
    total_tokens: int


class ChatCompletionChunk(_M):
    id: str
    object: Literal["chat.completion.chunk"]
    created: int
    model: str
    choices: List[Choice]
    usage: Optional[Usage] = None


def sdk_stream(text: str):
    """What openai-python's Stream does: split SSE events, stop at [DONE], JSON-decode, raise on error events."""
    for block in text.split("\n\n"):
        if not block.startswith("data: "):
            continue
        data = block[6:]
        if data == "[DONE]":
            return
        obj = json.loads(data)
        if "error" in obj:
            raise RuntimeError(obj["error"])
        yield ChatCompletionChunk.model_validate(obj)
    raise AssertionError("stream ended without [DONE]")


@pytest.fixture()
def client():
    llm = ScriptedProvider([{"tool_calls": [{"name": "count_slowly", "arguments": {"count": 2, "delay": 0}}]},
                            {"text": "all done here"}] * 4)
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=llm, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        yield c


@pytest.mark.parametrize("threaded", [False, True])
def test_stream_is_sdk_consumable(client, threaded):
    body = {"model": "kafka", "stream": True, "stream_options": {"include_usage": True},
            "messages": [{"role": "user", "content": "count then answer"}]}
    url = "/v1/threads/t-sdk/chat/completions" if threaded else "/v1/chat/completions"
    chunks = list(sdk_stream(client.post(url, json=body).text))
    text = "".join(c.choices[0].delta.content or "" for c in chunks if c.choices)
    assert text == "all done here"
    assert chunks[0].choices[0].delta.role == "assistant"
    finals = [c for c in chunks if c.choices and c.choices[0].finish_reason]
    assert finals and finals[-1].choices[0].finish_reason == "stop"
    assert chunks[-1].choices == [] and chunks[-1].usage is not None
    assert len({c.id for c in chunks}) == 1 and all(c.model == "kafka" for c in chunks)


def test_non_stream_matches_chat_completion_shape(client):
    r = client.post("/v1/chat/completions", json={"model": "kafka", "messages": [{"role": "user", "content": "x"}]})
    j = r.json()
    assert j["object"] == "chat.completion" and j["choices"][0]["message"]["content"] == "all done here"
    assert set(j["usage"]) >= {"prompt_tokens", "completion_tokens", "total_tokens"}
