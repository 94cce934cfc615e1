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
    xGMI all-reduce protocol at every layer seam, gloo control plane) serves /v1/threads/{id}/agent/run; the
    generation is constrained to a well-formed ``shell_exec`` call (random-init weights never emit one on their own),
    the call runs in the shipped sandbox service, its output streams back as tool_result frames, the loop ends with
    agent_done, and the assistant tool-call / tool messages are persisted (/root/reference/src/agents/base.py:372-433,
    /root/reference/server_tools/shell.py:14-75, /root/reference/src/kafka/base.py:229-310). The SSE transcript is
    written to $KAFKA_TRANSCRIPT_DIR when set (profiles/r03/config4_agent_run_sse.txt)."""
    import os
    import subprocess
    import sys

    import httpx

    monkeypatch.setenv("KAFKA_TP_BACKEND", "gloo")  # two ranks on one GPU: RCCL refuses, the custom AR does not
    port = _free_port()
    work = tmp_path / "sbx"
    work.mkdir()
    sbx = subprocess.Popen([sys.executable, "-m", "kafka_llm_service_amd.sandbox.service", "--port", str(port),
                            "--workdir", str(work)], env=dict(os.environ, HOME=str(tmp_path)))
    try:
        for _ in range(200):
            try:
                if httpx.get(f"http://127.0.0.1:{port}/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        cfg = ServerConfig(backend="engine", model="small-llama", tp=2, sandbox="shared",
                           sandbox_url=f"http://127.0.0.1:{port}", max_model_len=8192, prompt_sections=["intro"],
                           tool_choice={"type": "function", "function": {"name": "shell_exec"}},
                           agent_max_iterations=2, default_max_tokens=96,
                           engine_kwargs={"num_kv_blocks": 2048})
        st = ServerState(cfg, db=MemoryDBClient())
        with TestClient(create_app(state=st)) as c:
            assert c.get("/health").json()["kafka_initialized"]
            tid = c.post("/v1/threads").json()["thread_id"]
            r = c.post(f"/v1/threads/{tid}/agent/run",
                       json={"messages": [{"role": "user", "content": "List the files in the workspace."}],
                             "temperature": 0.7, "max_tokens": 96})
            text = r.text
            if os.environ.get("KAFKA_TRANSCRIPT_DIR"):
                with open(os.path.join(os.environ["KAFKA_TRANSCRIPT_DIR"], "config4_agent_run_sse.txt"), "w") as f:
                    f.write(text)
            fr = _frames(text)
            assert fr[-1] == "[DONE]"
            calls = [tc for x in fr if isinstance(x, dict) and x.get("choices")
                     for tc in (x["choices"][0]["delta"].get("tool_calls") or [])]
            assert any((tc.get("function") or {}).get("name") == "shell_exec" for tc in calls), calls[:3]
            results = [x for x in fr if isinstance(x, dict) and x.get("type") == "tool_result"]
            assert results and all(x["tool_name"] == "shell_exec" for x in results)
            assert any(x["is_complete"] for x in results)
            done = [x for x in fr if isinstance(x, dict) and x.get("type") == "agent_done"]
            assert done and done[-1]["reason"] == "max_iterations"
            msgs = c.get(f"/v1/threads/{tid}/messages").json()["messages"]
            roles = [m["role"] for m in msgs]
            assert roles[0] == "user" and "tool" in roles and "assistant" in roles
            tc_msgs = [m for m in msgs if m["role"] == "assistant" and m.get("tool_calls")]
            assert tc_msgs and tc_msgs[0]["tool_calls"][0]["function"]["name"] == "shell_exec"
            json.loads(tc_msgs[0]["tool_calls"][0]["function"]["arguments"])  # constrained: valid JSON arguments
    finally:
        sbx.terminate()
        sbx.wait(timeout=30)
