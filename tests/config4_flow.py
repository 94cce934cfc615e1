"""BASELINE config 4's tool-calling agent loop, shared by the CPU test (tests/test_constrained.py, tiny model) and
the GPU test (tests/test_server_gpu.py, a TP = 2 group on the MI355X).

A random-init model never emits a working call on its own, so the run pins it with the server's own knobs
(VERDICT r03 "Next round" #5): a per-iteration ``tool_choice`` script (iteration 1 ``create_shell``, 2 ``shell_exec``,
3 ``get_weather``) and ``enum`` schema overrides (``shell_id: main``, ``command: ls``, ``location: London``), so the
constrained decoder can only produce the calls of a real session: the shell is created, ``ls`` runs in the shipped
sandbox service and lists a file planted in its workdir, the weather tool answers from its offline fixtures, and the
second LLM call re-uses the first one's KV (usage events). Reference: /root/reference/server_tools/shell.py:14-75,
/root/reference/server_tools/weather.py:13-112, /root/reference/src/kafka/base.py:229-310.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

MARKER = "mi355x_marker_7f3a.txt"
SCRIPT = [{"type": "function", "function": {"name": n}} for n in ("create_shell", "shell_exec", "get_weather")]
OVERRIDES = {"create_shell": {"shell_id": {"type": "string", "enum": ["main"]}},
             "shell_exec": {"shell_id": {"type": "string", "enum": ["main"]},
                            "command": {"type": "string", "enum": ["ls"]}},
             "get_weather": {"location": {"type": "string", "enum": ["London"]}}}


def _frames(text: str) -> list:
    return [json.loads(b[6:]) for b in text.split("\n\n") if b.strip().startswith("data: {")]


def run(tmp_path, model: str, engine_kwargs: dict, sections: list[str] | None = ("intro",), on_done=None,
        **cfg_kw) -> tuple[str, list, list]:
    """Start a sandbox service + the API server, run one /v1/threads/{id}/agent/run turn; returns (SSE text,
    frames, persisted messages). ``sections=None``: the served default system prompt (the reference's 13 sections
    + the tool schemas, ~18k tokens)."""
    import httpx
    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    work = tmp_path / "sbx"
    work.mkdir()
    (work / MARKER).write_text("planted by the config-4 test\n")
    sbx = subprocess.Popen([sys.executable, "-m", "kafka_llm_service_amd.sandbox.service", "--port", str(port),
                            "--workdir", str(work)], env=dict(os.environ, HOME=str(tmp_path)))
    os.environ["KAFKA_WEATHER_MODE"] = "offline"
    try:
        for _ in range(300):
            try:
                if httpx.get(f"http://127.0.0.1:{port}/health", timeout=1).status_code == 200:
                    break
            except httpx.HTTPError:
                time.sleep(0.1)
        cfg = ServerConfig(backend="engine", model=model, sandbox="shared", sandbox_url=f"http://127.0.0.1:{port}",
                           tool_choice=SCRIPT, tool_overrides=OVERRIDES, agent_max_iterations=3,
                           prompt_sections=list(sections) if sections else None, engine_kwargs=engine_kwargs,
                           **cfg_kw)
        st = ServerState(cfg, db=MemoryDBClient())
        with TestClient(create_app(state=st)) as c:
            assert c.get("/health").json()["kafka_initialized"]
            tid = c.post("/v1/threads").json()["thread_id"]
            text = c.post(f"/v1/threads/{tid}/agent/run",
                          json={"messages": [{"role": "user", "content": "Create a shell, list the workspace, then "
                                                                          "check the weather in London."}],
                                "temperature": 0.7, "max_tokens": 96}).text
            msgs = c.get(f"/v1/threads/{tid}/messages").json()["messages"]
            if on_done is not None:
                on_done(c)
    finally:
        sbx.terminate()
        sbx.wait(timeout=30)
    return text, _frames(text), msgs


def check(text: str, frames: list, msgs: list) -> None:
    assert text.rstrip().endswith("data: [DONE]")
    calls = []
    for f in frames:
        for ch in f.get("choices") or []:
            for tc in ch["delta"].get("tool_calls") or []:
                if (tc.get("function") or {}).get("name"):
                    calls.append(tc["function"]["name"])
    assert calls == ["create_shell", "shell_exec", "get_weather"], calls
    res: dict[str, str] = {}
    for f in frames:
        if f.get("type") == "tool_result":
            res[f["tool_name"]] = res.get(f["tool_name"], "") + f["delta"]
    assert "does not exist" not in res["create_shell"] and "error" not in res["create_shell"].lower(), res
    assert MARKER in res["shell_exec"], res["shell_exec"]  # ls ran in the sandbox and listed the planted file
    assert "London" in res["get_weather"], res["get_weather"]
    usage = [f for f in frames if f.get("type") == "usage"]
    assert [u["iteration"] for u in usage] == [0, 1, 2]
    u1 = usage[1]["usage"]  # the second LLM call: system prompt + first call + its tool result are cached
    assert u1["cached_tokens"] >= 0.9 * u1["prompt_tokens"], u1
    done = [f for f in frames if f.get("type") == "agent_done"]
    assert done and done[-1]["reason"] == "max_iterations"
    roles = [m["role"] for m in msgs]
    assert roles == ["user", "assistant", "tool", "assistant", "tool", "assistant", "tool"], roles
    args = [json.loads(m["tool_calls"][0]["function"]["arguments"]) for m in msgs if m["role"] == "assistant"]
    assert args == [{"shell_id": "main"}, {"shell_id": "main", "command": "ls"}, {"location": "London"}], args
