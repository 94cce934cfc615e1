"""Schema-constrained tool-call decoding (engine/constrained.py): every path through the grammar is a well-formed
call that the tool-call parser accepts and that matches the tool's schema — for random token choices (fuzz), through
the engine (tiny random-init model), and through the agent loop of the HTTP server."""
import json
import random

import numpy as np
import pytest

from kafka_llm_service_amd.engine.chat_template import parse_tool_calls
from kafka_llm_service_amd.engine.constrained import Mask, ToolCallConstraint
from kafka_llm_service_amd.engine.tokenizer import get_tokenizer

TOOLS = [
    {"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "required": ["location", "days", "units", "tags", "deep", "opt"],
        "properties": {"location": {"type": "string"}, "days": {"type": "integer"},
                       "units": {"type": "string", "enum": ["c", "f"]}, "tags": {"type": "array",
                                                                             "items": {"type": "string"}},
                       "deep": {"type": "boolean"}, "opt": {"type": ["null", "number"], "minimum": 3, "maximum": 40},
                       "ignored": {"type": "string"}}}}},
    {"type": "function", "function": {"name": "get", "parameters": {"type": "object", "properties": {}}}},
    {"type": "function", "function": {"name": "idle", "parameters": {
        "type": "object", "properties": {"summary": {"type": "string"}}, "required": ["summary"]}}},
]


def _walk(c, rng, limit=400):
    out = []
    while len(out) < limit:
        spec = c(out)
        if spec is None:
            break
        ids = list(np.flatnonzero(spec.base)) + spec.extra if isinstance(spec, Mask) else list(spec)
        out.append(int(rng.choice(ids)))
    return out


@pytest.mark.parametrize("family", ["llama3", "mistral"])
def test_fuzz_required_calls_are_valid(family):
    tok = get_tokenizer(family, 128256 if family == "llama3" else 32000)
    for seed in range(30):
        c = ToolCallConstraint(tok, TOOLS, "required")
        out = _walk(c, random.Random(seed))
        assert c.done and out[0] == c.start and out[-1] == c.end
        calls = parse_tool_calls(tok.decode(out))
        assert calls and len(calls) == 1, tok.decode(out)
        fn = calls[0]["function"]
        args = json.loads(fn["arguments"])
        if fn["name"] == "get_weather":
            assert isinstance(args["location"], str) and isinstance(args["days"], int)
            assert args["units"] in ("c", "f") and isinstance(args["tags"], list) and len(args["tags"]) == 1
            assert isinstance(args["deep"], bool) and isinstance(args["opt"], (int, float))
            assert 3 <= args["opt"] <= 40
            assert "ignored" not in args
        elif fn["name"] == "idle":
            assert set(args) == {"summary"}
        else:
            assert fn["name"] == "get" and args == {}


def test_named_auto_and_none():
    tok = get_tokenizer("llama3")
    c = ToolCallConstraint(tok, TOOLS, {"type": "function", "function": {"name": "idle"}})
    out = _walk(c, random.Random(1))
    assert parse_tool_calls(tok.decode(out))[0]["function"]["name"] == "idle"
    # auto: unconstrained until the model opens a call, then the grammar applies
    a = ToolCallConstraint(tok, TOOLS, "auto")
    assert a([]) is None and a([5, 6]) is None
    a2 = ToolCallConstraint(tok, TOOLS, "auto")
    assert a2([]) is None and a2([a2.start]) is not None
    # none: the tool-call token is masked out of the first position
    n = ToolCallConstraint(tok, TOOLS, "none")
    m = n([])
    assert isinstance(m, Mask) and not m.base[n.start] and m.base[5]
    with pytest.raises(ValueError):
        ToolCallConstraint(tok, TOOLS, {"type": "function", "function": {"name": "nope"}})


def test_engine_forced_tool_call():
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams

    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048))
    tok = get_tokenizer("llama3")
    prompt = tok.encode("what is the weather in paris?")
    for temp in (0.0, 1.0):
        sp = SamplingParams(temperature=temp, max_tokens=200, ignore_eos=True, seed=3,
                            tool_grammar={"tools": TOOLS, "tool_choice": "required"})
        out = eng.generate([prompt], sp)[0]
        calls = parse_tool_calls(tok.decode(out))
        assert calls and out[-1] == tok.special_id("<|eom_id|>"), tok.decode(out)


def test_agent_loop_with_forced_idle_call():
    """/v1/agent/run on the real engine (tiny model, CPU): the forced call is executed and ends the loop."""
    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    cfg = ServerConfig(backend="engine", model="tiny-llama", sandbox="none", max_model_len=32768,
                       default_max_tokens=64, tool_choice={"type": "function", "function": {"name": "idle"}},
                       prompt_sections=["intro", "core_tools"],
                       engine_kwargs={"device": "cpu", "num_kv_blocks": 4096})
    st = ServerState(cfg, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        text = c.post("/v1/agent/run", json={"messages": [{"role": "user", "content": "wrap up"}]}).text
    frames = [json.loads(b[6:]) for b in text.split("\n\n") if b.startswith("data: {")]
    tr = [f for f in frames if f.get("type") == "tool_result"]
    assert tr and tr[0]["tool_name"] == "idle"
    done = [f for f in frames if f.get("type") == "agent_done"]
    assert done and done[0]["reason"] == "idle"


def test_agent_iterations_hit_the_prefix_cache(monkeypatch):
    """Iteration k+1 of the agent = iteration k + the assistant's tool-call tokens (re-emitted verbatim from the
    thread token cache) + the tool result, so only that suffix is prefilled (SURVEY.md §3.3 target)."""
    from fastapi.testclient import TestClient

    from kafka_llm_service_amd.db.local import MemoryDBClient
    from kafka_llm_service_amd.server.app import create_app
    from kafka_llm_service_amd.server.state import ServerConfig, ServerState

    monkeypatch.setenv("KAFKA_WEATHER_MODE", "offline")
    cfg = ServerConfig(backend="engine", model="tiny-llama", sandbox="none", max_model_len=32768,
                       default_max_tokens=48,
                       tool_choice={"type": "function", "function": {"name": "get_weather"}},
                       prompt_sections=["intro"], warm_prefix=False,
                       engine_kwargs={"device": "cpu", "num_kv_blocks": 4096})
    st = ServerState(cfg, db=MemoryDBClient())
    with TestClient(create_app(state=st)) as c:
        eng = st.engine_client.async_engine.engine
        seen = []
        orig = eng.add_request

        def spy(rid, prompt, params=None, meta=None):
            s = orig(rid, prompt, params, meta)
            seen.append(s)
            return s
        eng.add_request = spy
        st.kafka._agent.max_iterations = 3  # three forced weather calls, then max_iterations ends the run
        text = c.post("/v1/agent/run", json={"messages": [{"role": "user", "content": "weather?"}]}).text
    assert "get_weather" in text
    assert len(seen) >= 2
    for prev, cur in zip(seen, seen[1:]):
        # everything the previous iteration computed (its prompt and its generated call) is reused
        assert cur.num_cached >= (len(prev.prompt_ids) + len(prev.output_ids)) // 16 * 16 - 16, \
            (cur.num_cached, len(prev.prompt_ids), len(prev.output_ids))


def test_thread_agent_run_working_tools_against_sandbox_service(tmp_path):
    """Config 4's tool loop on CPU (tiny model): /v1/threads/{id}/agent/run with a per-iteration tool_choice script
    and enum schema overrides (tests/config4_flow.py) — create_shell, then ``ls`` in the shipped sandbox service
    listing a planted file, then the weather tool's offline fixture; the second LLM call hits the prefix cache; the
    tool turns are persisted. tests/test_server_gpu.py runs the same flow on a TP = 2 group on the GPU."""
    import config4_flow

    text, frames, msgs = config4_flow.run(tmp_path, "tiny-llama", {"device": "cpu", "num_kv_blocks": 4096},
                                          max_model_len=32768, default_max_tokens=96, warm_prefix=False)
    config4_flow.check(text, frames, msgs)
