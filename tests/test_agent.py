"""Agent loop, tool routing, compaction and KafkaAgent persistence with scripted (fake) LLMs (CPU, no network) —
the seams SURVEY.md §4.2 lists: a scripted LLMProvider, an in-memory DB, local tools."""
import asyncio
import json

from kafka_llm_service_amd.agents.base import Agent
from kafka_llm_service_amd.db.local import MemoryDBClient
from kafka_llm_service_amd.kafka.v1 import KafkaV1Provider, format_playbooks_table
from kafka_llm_service_amd.llm.compaction import (SummarizationCompactionProvider, TruncationCompactionProvider,
                                                  find_safe_split_point, is_context_length_error,
                                                  validate_message_structure)
from kafka_llm_service_amd.llm.stub import ScriptedProvider, StubEchoProvider
from kafka_llm_service_amd.llm.types import Message
from kafka_llm_service_amd.server_tools import PlannerTools, count_tool, get_weather_tool
from kafka_llm_service_amd.tools.agent import AgentToolProvider
from kafka_llm_service_amd.tools.types import Tool


def run(coro):
    return asyncio.run(coro)


async def collect(gen):
    return [e async for e in gen]


def _provider(**kw):
    tp = AgentToolProvider(tools=[count_tool, get_weather_tool], **kw)
    return tp


def test_text_response_events():
    llm = ScriptedProvider([{"text": "Hello there, friend!"}])
    tp = _provider()
    agent = Agent(llm, tp, system_prompt="SYS")
    evs = run(collect(agent.run([Message(role="user", content="hi")], model="m")))
    chunks = [e for e in evs if e.get("object") == "chat.completion.chunk"]
    assert chunks[0]["choices"][0]["delta"] == {"role": "assistant"}
    assert "".join(c["choices"][0]["delta"].get("content", "") for c in chunks) == "Hello there, friend!"
    assert chunks[-1]["choices"][0]["finish_reason"] == "stop"
    assert len({c["id"] for c in chunks}) == 1
    assert evs[-1]["type"] == "agent_done" and evs[-1]["reason"] == "text_response"
    assert evs[-1]["final_content"] == "Hello there, friend!" and evs[-1]["iteration"] == 0
    assert llm.calls[0][0].role == "system" and llm.calls[0][0].content == "SYS"  # system prompt prepended


def test_tool_call_then_idle():
    llm = ScriptedProvider([
        {"tool_calls": [{"name": "count_slowly", "arguments": {"count": 3, "delay": 0}}]},
        {"text": "counted", "tool_calls": [{"name": "idle", "arguments": {"summary": "done counting"}}]},
    ])
    agent = Agent(llm, _provider())
    evs = run(collect(agent.run([Message(role="user", content="count")], model="m")))
    tr = [e for e in evs if e.get("type") == "tool_result"]
    count_deltas = [e["delta"] for e in tr if e["tool_name"] == "count_slowly"]
    assert "".join(count_deltas) == "1... 2... 3... Done!"
    assert tr[len(count_deltas) - 1]["is_complete"] and tr[len(count_deltas) - 1]["delta"] == ""
    idle = [e for e in tr if e["tool_name"] == "idle"]
    assert idle and json.loads(idle[0]["delta"]) == {"status": "idle", "summary": "done counting"}
    assert evs[-1] == {"type": "agent_done", "reason": "idle", "summary": "done counting", "iteration": 1,
                       "usage": evs[-1]["usage"]}
    # the second LLM call saw the assistant tool call and the tool result
    roles = [m.role for m in llm.calls[1]]
    assert roles[-2:] == ["assistant", "tool"] and llm.calls[1][-1].content == "1... 2... 3... Done!"
    # chunk ids differ per iteration
    ids = [e["id"] for e in evs if e.get("object")]
    assert len(set(ids)) == 2


def test_unknown_tool_bad_json_and_max_iterations():
    llm = ScriptedProvider([{"tool_calls": [{"name": "nope", "arguments": "{not json"}]}] * 3)
    agent = Agent(llm, _provider(), max_iterations=3)
    evs = run(collect(agent.run([Message(role="user", content="x")], model="m")))
    errs = [e for e in evs if e.get("type") == "tool_result"]
    assert errs[0]["delta"] == "Error: Tool not found: nope" and errs[0]["is_complete"]
    assert evs[-1]["reason"] == "max_iterations" and evs[-1]["iteration"] == 3


def test_tool_order_is_stable_and_idle_appended():
    tp = AgentToolProvider(tools=[get_weather_tool, count_tool] + PlannerTools("t").tools)
    Agent(StubEchoProvider(), tp)
    names = [t["function"]["name"] for t in run(tp.get_tools())]
    assert names == ["get_weather", "count_slowly", "sequentialthinking", "saveThoughtCheckpoint",
                     "loadThoughtCheckpoint", "idle"]


def test_context_compaction_retry():
    err = "This model's maximum context length is 100 tokens. However, your messages resulted in 150 tokens."
    llm = ScriptedProvider([{"error": err}, {"text": "after compaction"}])
    msgs = [Message(role="user" if i % 2 == 0 else "assistant", content=f"m{i}") for i in range(60)]
    agent = Agent(llm, _provider(), system_prompt="S", context_compaction_provider=TruncationCompactionProvider(10))
    evs = run(collect(agent.run(msgs, model="m")))
    assert evs[-1]["reason"] == "text_response" and evs[-1]["final_content"] == "after compaction"
    assert len(llm.calls[-1]) == 11  # system + last 10


def test_summarization_compaction_uses_llm_and_string_content():
    summarizer = ScriptedProvider([{"text": "SUMMARY"}])
    comp = SummarizationCompactionProvider(summarizer, min_messages_to_summarize=4)
    msgs = [{"role": "system", "content": "S"}] + [{"role": "user", "content": f"u{i}"} for i in range(8)]
    out = run(comp.compact(msgs, "S", "m"))
    assert out[0]["content"] == "S"
    assert out[1]["role"] == "system" and isinstance(out[1]["content"], str) and "SUMMARY" in out[1]["content"]
    assert [m["content"] for m in out[2:]] == ["u6", "u7"]


def test_compaction_helpers():
    assert is_context_length_error(Exception("context_length_exceeded"))
    assert is_context_length_error(Exception("prompt is too long: 200 tokens > 100"))
    assert not is_context_length_error(Exception("rate limit"))
    msgs = [{"role": "user"}, {"role": "assistant", "tool_calls": [{"id": "a"}]}, {"role": "tool", "tool_call_id": "a"},
            {"role": "user"}]
    assert find_safe_split_point(msgs, 2) == 1 and find_safe_split_point(msgs, 3) == 3
    v = validate_message_structure([{"role": "tool", "tool_call_id": "zz"}, {"role": "assistant"},
                                    {"role": "user", "content": "x"}])
    assert v == [{"role": "user", "content": "x"}]


def test_planner_state_is_per_thread():
    a, b = PlannerTools("thread-a"), PlannerTools("thread-b")
    run(a.tools[0].run({"thought": "t1", "nextThoughtNeeded": True, "thoughtNumber": 1, "totalThoughts": 2,
                        "goalSummary": "goal A"}))
    res = json.loads(run(b.tools[0].run({"thought": "x", "nextThoughtNeeded": False, "thoughtNumber": 1,
                                         "totalThoughts": 1})))
    assert res["thoughtHistoryLength"] == 1 and res["goalSummary"] == ""
    json.loads(run(a.tools[1].run({"checkpointId": "c1"})))
    out = json.loads(run(a.tools[2].run({"checkpointId": "c1"})))
    assert out["goalSummary"] == "goal A"


def test_kafka_v1_thread_persistence_and_profile_prompt():
    async def main():
        db = MemoryDBClient()
        await db.initialize()
        await db.upsert_kafka_profile("p1", global_prompt="ALWAYS BE BRIEF")
        await db.add_playbook("p1", "Deploy | prod", "When shipping\nto prod")
        t = await db.create_thread(kafka_profile_id="p1")
        llm = ScriptedProvider([
            {"tool_calls": [{"name": "get_weather", "arguments": {"location": "Paris"}}]},
            {"text": "It is nice."},
        ])
        k = KafkaV1Provider(llm, thread_id=t["id"], db_client=db, tools=[get_weather_tool])
        await k.initialize()
        assert "ALWAYS BE BRIEF" in k.system_prompt and "| Deploy \\| prod | When shipping to prod |" in \
            k.system_prompt
        assert k.system_prompt.index("ALWAYS BE BRIEF") < k.system_prompt.index("Available Playbooks")
        evs = await collect(k.run_with_thread([Message(role="user", content="weather?")], model="m"))
        assert evs[-1]["final_content"] == "It is nice."
        assert all(e.get("type") != "_message" for e in evs)
        hist = await db.get_thread_messages(t["id"])
        assert [m.role for m in hist] == ["user", "assistant", "tool", "assistant"]
        assert hist[1].tool_calls[0]["function"]["name"] == "get_weather"
        assert hist[2].tool_call_id == hist[1].tool_calls[0]["id"] and "Weather in Paris" in hist[2].content
        assert hist[3].content == "It is nice."
        await k.cleanup()
    import os
    os.environ["KAFKA_WEATHER_MODE"] = "offline"
    run(main())


def test_playbooks_table_empty():
    assert format_playbooks_table([]) == ""


def test_tool_handlers_sync_async_stream():
    async def agen(n: int):
        for i in range(n):
            yield str(i)

    t1 = Tool("a", "", {}, handler=lambda x: {"x": x})
    t2 = Tool("b", "", {}, handler=agen)
    assert run(t1.run({"x": 1})) == {"x": 1}
    assert run(t2.run({"n": 3})) == "012"
    assert run(collect(t1.run_stream({"x": 2}))) == ['{"x": 2}']
    assert t2.is_streaming and not t1.is_streaming


def test_reference_prompt_renders_byte_identically(monkeypatch):
    """The served default system prompt is the reference's text (prompts/sections_reference, shipped as data per
    SURVEY.md §2.1 #18): with the default enrichment (/root/reference/src/prompts/v1.py:73-117) it renders to
    exactly the reference's 70,496-char prompt (sha256 of the reference rendering, computed from its section files
    with its substitution rule and "\\n\\n" separator). KAFKA_PROMPT=compact selects this repo's shorter wording."""
    import hashlib

    from kafka_llm_service_amd.prompts.v1 import PromptProviderV1

    monkeypatch.delenv("KAFKA_PROMPT", raising=False)
    text = PromptProviderV1().get_system_prompt()
    assert len(text) == 70496
    assert hashlib.sha256(text.encode()).hexdigest() == \
        "6feb95e05419a8fbc97c5ad110d7b06c5b2227715304b9a5c10b825876283cf7"
    assert PromptProviderV1(variant="reference").get_system_prompt() == text
    compact = PromptProviderV1(variant="compact").get_system_prompt()
    assert 40000 < len(compact) < 60000 and compact != text
    monkeypatch.setenv("KAFKA_PROMPT", "compact")
    assert PromptProviderV1().get_system_prompt() == compact
    # the minimal / tools-only derivatives keep the variant's text
    minimal = PromptProviderV1(variant="reference").create_minimal().get_system_prompt()
    assert text.startswith(minimal.split("\n\n---")[0]) and len(minimal) < len(text)
