"""The HTTP API on the MI355X: engine in its own worker process (the GPU default), live token streaming with usage,
the pinned shared system prefix reused by a new thread, thread history persisted."""
import json
import time

import pytest
from fastapi.testclient import TestClient

from kafka_llm_service_amd.db.local import MemoryDBClient
from kafka_llm_service_amd.server.app import create_app
from kafka_llm_service_amd.server.state import ServerConfig, ServerState

pytestmark = pytest.mark.gpu


def _frames(text):
    out = []
    for block in text.split("\n\n"):
        block = block.strip()
        if block:
            payload = block[6:]
            out.append(payload if payload == "[DONE]" else json.loads(payload))
    return out


@pytest.mark.timeout(300)
def test_threaded_chat_over_http_with_engine_process(cuda):
    cfg = ServerConfig(backend="engine", model="small-llama", sandbox="none", max_model_len=8192,
                       prompt_sections=["intro", "core_tools"], engine_process=True, ignore_eos=True,
                       engine_kwargs={"num_kv_blocks": 4096})
    st = ServerState(cfg, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        assert c.get("/health").json()["kafka_initialized"]
        tid = c.post("/v1/threads").json()["thread_id"]
        body = {"model": "small-llama", "messages": [{"role": "user", "content": "Hello MI355X"}], "stream": True,
                "temperature": 0, "max_tokens": 12, "stream_options": {"include_usage": True}}
        f = _frames(c.post(f"/v1/threads/{tid}/chat/completions", json=body).text)
        assert f[-1] == "[DONE]"
        content = [x for x in f if isinstance(x, dict) and x.get("choices") and x["choices"][0]["delta"].get("content")]
        assert len(content) >= 2  # live token frames, not one post-hoc blob
        usage = [x for x in f if isinstance(x, dict) and x.get("usage")][0]["usage"]
        assert usage["completion_tokens"] == 12 and usage["prompt_tokens"] > 100
        health = {}
        for _ in range(50):  # the worker answers health requests asynchronously
            health = st.engine_client.health()["replica0"]
            if "prefix_hit_tokens" in health:
                break
            time.sleep(0.05)
        assert health["prefix_hit_tokens"] >= usage["prompt_tokens"] - 64  # pinned system prefix reused
        body["messages"] = [{"role": "user", "content": "And the HBM?"}]
        body["stream"] = False
        r = c.post(f"/v1/threads/{tid}/chat/completions", json=body).json()
        assert r["usage"]["completion_tokens"] == 12
        msgs = c.get(f"/v1/threads/{tid}/messages").json()["messages"]
        assert [m["role"] for m in msgs] == ["user", "assistant", "user", "assistant"]


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_config4_agent_tool_loop_tp2_with_sandbox_service(cuda, tmp_path, monkeypatch):
    """BASELINE config 4 end to end on one MI355X: a TP=2 engine group (two worker processes on the one GPU: custom
    xGMI all-reduce protocol at every layer seam, gloo control plane) serves /v1/threads/{id}/agent/run and the
    agent loop runs WORKING tools (tests/config4_flow.py): create_shell, then ``ls`` in the shipped sandbox service
    (its output lists a file planted in the workdir), then get_weather on a fixture city; the second LLM call hits
    the prefix cache for >= 90 % of its prompt; the tool turns are persisted (/root/reference/src/agents/base.py:
    372-433, /root/reference/server_tools/shell.py:14-75, /root/reference/src/kafka/base.py:229-310). The SSE
    transcript is written to $KAFKA_TRANSCRIPT_DIR when set (profiles/r04/config4_agent_run_sse.txt)."""
    import os

    import config4_flow

    monkeypatch.setenv("KAFKA_TP_BACKEND", "gloo")  # two ranks on one GPU: RCCL refuses, the custom AR does not
    text, frames, msgs = config4_flow.run(tmp_path, "small-llama", {"num_kv_blocks": 2048}, tp=2, max_model_len=8192,
                                          default_max_tokens=96)
    if os.environ.get("KAFKA_TRANSCRIPT_DIR"):
        with open(os.path.join(os.environ["KAFKA_TRANSCRIPT_DIR"], "config4_agent_run_sse.txt"), "w") as f:
            f.write(text)
    config4_flow.check(text, frames, msgs)
