"""HTTP contract tests for every route (SURVEY.md §2.5, §4.3 golden-trace method): frame order, key sets, explicit
nulls, [DONE], error frames, 404/422 — against the stub echo provider (BASELINE config 1) and, end to end, against
the real engine on a tiny random-init model on CPU (live token streaming, usage, prefix-cache hits across turns)."""
import json

import pytest
from fastapi.testclient import TestClient

from kafka_llm_service_amd.db.local import MemoryDBClient
from kafka_llm_service_amd.llm.stub import ScriptedProvider
from kafka_llm_service_amd.server.app import create_app
from kafka_llm_service_amd.server.state import ServerConfig, ServerState


def frames(text):
    out = []
    for block in text.split("\n\n"):
        block = block.strip()
        if not block:
            continue
        assert block.startswith("data: ")
        payload = block[6:]
        out.append(payload if payload == "[DONE]" else json.loads(payload))
    return out


@pytest.fixture()
def stub_client():
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        yield c


def test_thread_crud(stub_client):
    c = stub_client
    r = c.post("/v1/threads", json={"system_message": "be nice", "user_id": "u1"})
    tid = r.json()["thread_id"]
    assert set(r.json()) == {"thread_id", "created_at"}
    assert c.post(f"/v1/threads/{tid}/messages", json={"role": "user", "content": "hi"}).json()["success"]
    msgs = c.get(f"/v1/threads/{tid}/messages").json()
    assert msgs["thread_id"] == tid and msgs["messages"] == [{"role": "system", "content": "be nice"},
                                                               {"role": "user", "content": "hi"}]
    assert c.delete(f"/v1/threads/{tid}/messages").json() == {"success": True, "deleted_count": 2}
    assert c.get("/v1/threads/nope/messages").status_code == 404
    assert c.delete("/v1/threads/nope/messages").status_code == 404
    assert c.post("/v1/threads").status_code == 200  # body optional
    # auto-create on POST message
    assert c.post("/v1/threads/auto1/messages", json={"role": "user", "content": "x"}).json()["success"]
    assert c.get("/v1/threads/auto1/messages").status_code == 200


def test_validation_errors(stub_client):
    r = stub_client.post("/v1/chat/completions", json={"model": "m", "messages": [], "temperature": 3})
    assert r.status_code == 422
    r = stub_client.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "x"}]})
    assert r.status_code == 422


def test_thread_chat_stream_grammar(stub_client):
    c = stub_client
    tid = c.post("/v1/threads").json()["thread_id"]
    r = c.post(f"/v1/threads/{tid}/chat/completions", json={
        "model": "my-model", "messages": [{"role": "user", "content": "hello"}], "stream": True,
        "stream_options": {"include_usage": True}})
    assert r.headers["content-type"].startswith("text/event-stream")
    assert r.headers["cache-control"] == "no-cache" and r.headers["x-accel-buffering"] == "no"
    f = frames(r.text)
    assert f[-1] == "[DONE]"
    first = f[0]
    assert first["object"] == "chat.completion.chunk" and first["model"] == "my-model"
    assert first["choices"] == [{"index": 0, "delta": {"role": "assistant", "content": None, "tool_calls": None},
                                 "finish_reason": None}]
    assert first["id"].startswith("chatcmpl-") and len(first["id"]) == len("chatcmpl-") + 24
    content = [x for x in f[1:-1] if isinstance(x, dict) and x.get("choices") and
               x["choices"][0]["delta"]["content"]]
    assert "".join(x["choices"][0]["delta"]["content"] for x in content).startswith("hello")
    stop = [x for x in f if isinstance(x, dict) and x.get("choices") and x["choices"][0]["finish_reason"]]
    assert stop[-1]["choices"][0]["finish_reason"] == "stop"
    usage = [x for x in f if isinstance(x, dict) and "usage" in x]
    assert usage and usage[0]["choices"] == [] and usage[0]["usage"]["completion_tokens"] == 128
    assert len({x["id"] for x in f if isinstance(x, dict)}) == 1
    # the reply was persisted after the user message
    msgs = c.get(f"/v1/threads/{tid}/messages").json()["messages"]
    assert [m["role"] for m in msgs] == ["user", "assistant"]


def test_non_stream_has_usage(stub_client):
    r = stub_client.post("/v1/chat/completions", json={"model": "m", "messages": [{"role": "user", "content": "ab"}]})
    j = r.json()
    assert j["object"] == "chat.completion" and j["choices"][0]["message"]["role"] == "assistant"
    assert j["choices"][0]["finish_reason"] == "stop"
    assert j["usage"]["completion_tokens"] == 128 and j["usage"]["total_tokens"] > 128


def test_models_health_metrics(stub_client):
    assert stub_client.get("/v1/models").json()["object"] == "list"
    h = stub_client.get("/health").json()
    assert h["status"] == "healthy" and h["kafka_initialized"] is True
    stub_client.post("/v1/chat/completions", json={"model": "m", "messages": [{"role": "user", "content": "x"}],
                                                   "stream": True})
    m = stub_client.get("/metrics").text
    assert "kafka_requests_total" in m and "kafka_ttft_seconds_bucket" in m


def test_agent_run_tool_events_and_error_frame():
    llm = ScriptedProvider([{"tool_calls": [{"name": "count_slowly", "arguments": {"count": 2, "delay": 0}}]},
                            {"text": "done", "tool_calls": [{"name": "idle", "arguments": {"summary": "ok"}}]},
                            {"error": "boom"}])
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=llm, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        f = frames(c.post("/v1/agent/run", json={"messages": [{"role": "user", "content": "go"}]}).text)
        types = [x.get("type") if isinstance(x, dict) else x for x in f]
        assert "tool_result" in types and f[-1] == "[DONE]"
        done = [x for x in f if isinstance(x, dict) and x.get("type") == "agent_done"][0]
        assert done["reason"] == "idle" and done["summary"] == "ok"
        tr = [x for x in f if isinstance(x, dict) and x.get("type") == "tool_result"]
        assert set(tr[0]) == {"type", "tool_call_id", "tool_name", "delta", "is_complete"}
        f2 = frames(c.post("/v1/agent/run", json={"messages": [{"role": "user", "content": "go"}]}).text)
        assert f2[-2]["error"]["type"] == "agent_error" and f2[-1] == "[DONE]"


def test_chat_completions_tool_events_opt_in():
    def script():
        return [{"tool_calls": [{"name": "count_slowly", "arguments": {"count": 1, "delay": 0}}]}, {"text": "fin"}]
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=ScriptedProvider(script() * 2),
                     db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        body = {"model": "m", "messages": [{"role": "user", "content": "x"}], "stream": True}
        plain = frames(c.post("/v1/chat/completions", json=body).text)
        assert all("choices" in x for x in plain if isinstance(x, dict))  # OpenAI-SDK-safe by default
        opted = frames(c.post("/v1/chat/completions", json=body, headers={"X-Kafka-Tool-Events": "1"}).text)
        assert any(isinstance(x, dict) and x.get("type") == "tool_result" for x in opted)


def test_thread_agent_run_persists(tmp_path):
    llm = ScriptedProvider([{"tool_calls": [{"name": "get_weather", "arguments": {"location": "Tokyo"}}]},
                            {"text": "sunny"}])
    import os
    os.environ["KAFKA_WEATHER_MODE"] = "offline"
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=llm, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        f = frames(c.post("/v1/threads/t-agent/agent/run",
                          json={"messages": [{"role": "user", "content": "weather in tokyo"}]}).text)
        assert f[-1] == "[DONE]"
        msgs = c.get("/v1/threads/t-agent/messages").json()["messages"]
        assert [m["role"] for m in msgs] == ["user", "assistant", "tool", "assistant"]
        assert "Tokyo" in msgs[2]["content"] and msgs[3]["content"] == "sunny"


# ---------------------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def engine_client():
    st = ServerState(ServerConfig(backend="engine", model="tiny-llama", sandbox="none", max_model_len=8192,
                                  default_max_tokens=12, prompt_sections=["intro", "core_principles", "core_tools"],
                                  engine_kwargs={"device": "cpu", "num_kv_blocks": 1024}),
                     db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        yield c, st


def test_engine_streaming_and_prefix_reuse(engine_client):
    c, st = engine_client
    tid = c.post("/v1/threads").json()["thread_id"]
    body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "Tell me about MI355X."}],
            "stream": True, "temperature": 0, "max_tokens": 8, "stream_options": {"include_usage": True}}
    f1 = frames(c.post(f"/v1/threads/{tid}/chat/completions", json=body).text)
    assert f1[-1] == "[DONE]"
    u1 = [x for x in f1 if isinstance(x, dict) and "usage" in x][0]["usage"]
    assert u1["completion_tokens"] >= 1 and u1["prompt_tokens"] > 100  # Kafka system prompt + tools rendered
    # the shared system prefix was prefilled and pinned at start-up: even turn 1 of a new thread is a prefix hit
    h0 = st.engine_client.health()["replica0"]
    assert h0["prefix_hit_tokens"] >= u1["prompt_tokens"] - 64
    body["messages"] = [{"role": "user", "content": "And its HBM?"}]
    c.post(f"/v1/threads/{tid}/chat/completions", json=body)
    h = st.engine_client.health()["replica0"]
    # turn 2 re-used the shared system prefix and turn 1's history from the prefix cache
    assert h["prefix_hit_tokens"] >= u1["prompt_tokens"] - 16
    msgs = c.get(f"/v1/threads/{tid}/messages").json()["messages"]
    assert [m["role"] for m in msgs] == ["user", "assistant", "user", "assistant"]


def test_engine_context_length_error(engine_client):
    c, _ = engine_client
    body = {"model": "tiny-llama", "messages": [{"role": "user", "content": "word " * 9000}], "stream": True,
            "max_tokens": 4}
    f = frames(c.post("/v1/chat/completions", json=body).text)
    err = [x for x in f if isinstance(x, dict) and "error" in x]
    assert err and "maximum context length" in err[0]["error"]["message"] and f[-1] == "[DONE]"


def test_engine_unavailable_is_503():
    """A dead / restarting engine replica surfaces as HTTP 503 on non-stream requests (retryable) and as an error
    frame on streams."""
    from kafka_llm_service_amd.engine.client import EngineUnavailable
    from kafka_llm_service_amd.llm.base import LLMProvider

    class Down(LLMProvider):
        async def stream_completion(self, messages, **kw):
            raise EngineUnavailable("engine replica 0 is down")
            yield  # pragma: no cover

        async def completion(self, messages, **kw):
            raise EngineUnavailable("engine replica 0 is down")

    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=Down(), db=MemoryDBClient())
    with TestClient(create_app(state=st), raise_server_exceptions=False) as c:
        body = {"model": "kafka", "messages": [{"role": "user", "content": "hi"}]}
        r = c.post("/v1/chat/completions", json=body)
        assert r.status_code == 503 and "down" in r.json()["detail"]
        r = c.post("/v1/chat/completions", json=dict(body, stream=True))
        fr = frames(r.text)
        assert fr[-1] == "[DONE]" and "error" in fr[-2]
