"""Observability: Chrome-trace spans of engine phases / requests / tools when
KAFKA_TRACE_FILE is set, and the Prometheus histograms the server exports."""
import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path


def test_trace_file_has_engine_and_request_spans(tmp_path):
    code = textwrap.dedent("""
        from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
        from kafka_llm_service_amd.engine.sequence import SamplingParams
        from kafka_llm_service_amd.obs import trace
        e = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_kv_blocks=128, max_model_len=1024))
        e.generate([list(range(100, 130)), list(range(200, 220))],
                   SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
        trace.tracer().close()
    """)
    env = dict(os.environ, KAFKA_TRACE_FILE=str(tmp_path / "tr"),
               PYTHONPATH=str(Path(__file__).resolve().parents[1]))
    subprocess.run([sys.executable, "-c", code], check=True, env=env, timeout=300)
    files = list(tmp_path.glob("tr.*.json"))
    assert len(files) == 1
    evs = [e for e in json.loads(files[0].read_text()) if e]
    names = {e["name"] for e in evs}
    assert {"schedule", "launch", "collect", "request", "first_token", "decode"} <= names
    req = [e for e in evs if e["name"] == "request"]
    assert len(req) == 2 and all(e["args"]["output_tokens"] == 4 and e["dur"] > 0 for e in req)


def test_metrics_histograms_exported():
    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.llm.stub import ScriptedProvider
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    llm = ScriptedProvider([{"tool_calls": [{"name": "count_slowly", "arguments": {"count": 1, "delay": 0}}]},
                            {"text": "done and dusted"}])
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=llm, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        c.post("/v1/chat/completions", json={"model": "m", "messages": [{"role": "user", "content": "x"}],
                                             "stream": True, "stream_options": {"include_usage": True}})
        m = c.get("/metrics").text
    import re

    cnt = re.search(r'kafka_tool_seconds_count\{tool="count_slowly"\} ([0-9.]+)', m)
    assert cnt and float(cnt.group(1)) >= 1
    assert "kafka_tpot_seconds_bucket" in m and "kafka_output_tokens_total" in m


def test_agent_run_feeds_serving_metrics():
    """/v1/threads/{id}/agent/run observes TTFT / end-to-end time and counts its output tokens, as the chat route."""
    import re

    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.llm.stub import ScriptedProvider
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    def grab(m, name):
        x = re.search(rf"^{name} ([0-9.e+]+)$", m, re.M)
        return float(x.group(1)) if x else 0.0

    llm = ScriptedProvider([{"text": "all done here"}])
    st = ServerState(ServerConfig(backend="stub", sandbox="none"), llm_provider=llm, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        m0 = c.get("/metrics").text
        tid = c.post("/v1/threads").json()["thread_id"]
        body = c.post(f"/v1/threads/{tid}/agent/run", json={"messages": [{"role": "user", "content": "hi"}]}).text
        m1 = c.get("/metrics").text
    assert body.rstrip().endswith("data: [DONE]")
    assert grab(m1, "kafka_ttft_seconds_count") == grab(m0, "kafka_ttft_seconds_count") + 1
    assert grab(m1, "kafka_request_seconds_count") == grab(m0, "kafka_request_seconds_count") + 1
    assert grab(m1, "kafka_output_tokens_total") > grab(m0, "kafka_output_tokens_total")


def test_json_logging_lines():
    import io
    import logging

    from kafka_llm_service_amd.obs.logging import setup_logging

    buf = io.StringIO()
    setup_logging(json_lines=True, level="INFO", stream=buf)
    logging.getLogger("kafka.engine").info("step done", extra={"step": 7, "ms": 9.4})
    rec = json.loads(buf.getvalue().strip().splitlines()[-1])
    assert rec["msg"] == "step done" and rec["step"] == 7 and rec["level"] == "INFO" and rec["logger"] == "kafka.engine"
    setup_logging(json_lines=False, stream=io.StringIO())


def test_server_cli_flags_map_to_config(monkeypatch):
    from kafka_llm_service_amd.server import __main__ as m
    from kafka_llm_service_amd.server.state import ServerConfig

    for env in m.FLAGS.values():
        monkeypatch.delenv(env, raising=False)
    monkeypatch.setenv("KAFKA_MODEL", "tiny-llama")
    monkeypatch.setenv("KAFKA_DP", "2")
    monkeypatch.setenv("KAFKA_PROMPT_SECTIONS", "intro,core_tools")
    cfg = ServerConfig.from_env()
    assert cfg.model == "tiny-llama" and cfg.dp == 2 and cfg.prompt_sections == ["intro", "core_tools"]


def test_metrics_per_gpu_step_time():
    """/metrics carries each replica's GPU step time (and collective time when the replica has an IPC
    collective; the GPU TP tests cover that path) labelled by replica and device."""
    import re

    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    cfg = ServerConfig(backend="engine", model="tiny-llama", sandbox="none", max_model_len=4096, warm_prefix=False,
                       prompt_sections=["intro"], ignore_eos=True, engine_kwargs={"device": "cpu", "num_kv_blocks": 512})
    st = ServerState(cfg, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        c.post("/v1/chat/completions", json={"model": "m", "messages": [{"role": "user", "content": "x"}],
                                             "max_tokens": 12, "temperature": 0})
        m = ""
        for _ in range(50):
            m = c.get("/metrics").text
            if "kafka_gpu_step_ms" in m:
                break
    v = re.search(r'kafka_gpu_step_ms\{replica="0",device="cpu",stat="p50"\} ([0-9.]+)', m)
    assert v and float(v.group(1)) > 0, m[-2000:]
