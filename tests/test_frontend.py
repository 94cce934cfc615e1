"""Tokenizer / chat template / tool-call parsing: the prefix-stability property the prefix cache depends on
 and the OpenAI tool_calls shape (portkey.py:447-464 normalisation)."""
import json

from hypothesis import given, settings, strategies as st

from kafka_llm_service_amd.engine.chat_template import ChatTemplate, parse_tool_calls
from kafka_llm_service_amd.engine.tokenizer import IncrementalDetokenizer, get_tokenizer
from kafka_llm_service_amd.llm.types import Message
from kafka_llm_service_amd.server_tools import count_tool, get_weather_tool

TOK = get_tokenizer("llama3", 128256)
TPL = ChatTemplate(TOK)
TOOLS = [get_weather_tool.definition, count_tool.definition]

texts = st.text(alphabet=st.characters(blacklist_categories=("Cs",)), min_size=0, max_size=40)
msgs = st.lists(st.tuples(st.sampled_from(["user", "assistant", "tool"]), texts), min_size=1, max_size=6)


@settings(max_examples=80, deadline=None)
@given(msgs, texts)
def test_history_render_is_token_prefix(history, new_text):
    hist = [Message(role="system", content="SYS")] + [
        Message(role=r, content=t, tool_call_id="c1" if r == "tool" else None) for r, t in history]
    a = TPL.render(hist, TOOLS, add_generation_prompt=False)
    b = TPL.render(hist + [Message(role="user", content=new_text)], TOOLS)
    assert b[:len(a)] == a


def test_generated_tokens_reused_verbatim():
    prompt_msgs = [Message(role="system", content="S"), Message(role="user", content="q")]
    p = TPL.render(prompt_msgs, TOOLS)
    gen = [500, 70000, 91234, TOK.special_id("<|eot_id|>")]  # arbitrary ids + eot
    hist = prompt_msgs + [Message(role="assistant", content=TOK.decode(gen), token_ids=gen)]
    nxt = TPL.render(hist + [Message(role="user", content="more")], TOOLS)
    assert nxt[:len(p) + len(gen)] == p + gen


def test_special_tokens_and_roundtrip():
    ids = TOK.encode("Hello, MI355X world!")
    assert TOK.decode(ids) == "Hello, MI355X world!"
    assert TOK.decode([TOK.special_id("<|eot_id|>")]) == ""
    assert TOK.decode([TOK.special_id("<|eot_id|>")], skip_special_tokens=False) == "<|eot_id|>"
    assert TOK.decode([120000]).strip()  # a high regular id decodes to text
    d = IncrementalDetokenizer(TOK)
    s = "".join(d.add([i]) for i in TOK.encode("héllo wörld ✓ done"))
    assert s == "héllo wörld ✓ done"


def test_tool_call_render_and_parse():
    m = Message(role="assistant", tool_calls=[{"id": "a", "type": "function",
                                               "function": {"name": "get_weather", "arguments": '{"location":"X"}'}}])
    ids = TPL.render_message(m)
    assert TOK.special_id("<|python_tag|>") in ids
    body = TOK.decode(ids[ids.index(TOK.special_id("<|python_tag|>")) + 1:])
    calls = parse_tool_calls(body)
    assert calls[0]["function"]["name"] == "get_weather"
    assert json.loads(calls[0]["function"]["arguments"]) == {"location": "X"}
    assert calls[0]["type"] == "function" and calls[0]["id"].startswith("call_") and calls[0]["index"] == 0
    two = parse_tool_calls('{"name": "a", "parameters": {}}\n{"name": "b", "parameters": {"x": 1}}')
    assert [c["function"]["name"] for c in two] == ["a", "b"] and two[1]["index"] == 1
    assert parse_tool_calls("not a call") is None


def test_mistral_template():
    tok = get_tokenizer("mistral", 32000)
    tpl = ChatTemplate(tok)
    ids = tpl.render([Message(role="user", content="hi")], TOOLS)
    assert ids[0] == 1 and tok.special_id("[INST]") in ids and tok.special_id("[AVAILABLE_TOOLS]") in ids
    assert tok.decode(tok.encode("abc def")) == "abc def"


def test_local_db_opens_a_reference_schema_database(tmp_path):
    """A threads.db written by the reference (its SQLite schema, same-second created_at ties, multi-part content)
    opens in place: history comes back in insertion order, new messages append after it."""
    import asyncio
    import sqlite3

    from kafka_llm_service_amd.db.local import LocalDBClient

    path = tmp_path / "threads.db"
    c = sqlite3.connect(path)
    c.executescript("""
        CREATE TABLE threads (id TEXT PRIMARY KEY, created_at TEXT DEFAULT CURRENT_TIMESTAMP, metadata TEXT,
                              sandbox_id TEXT);
        CREATE TABLE messages (id TEXT PRIMARY KEY, thread_id TEXT NOT NULL, message TEXT NOT NULL, metadata TEXT,
                               created_at TEXT DEFAULT CURRENT_TIMESTAMP, FOREIGN KEY (thread_id) REFERENCES threads(id));
        CREATE INDEX idx_messages_thread_id ON messages(thread_id);""")
    c.execute("INSERT INTO threads(id, created_at, metadata) VALUES ('t1', '2025-01-01 10:00:00', '{}')")
    msgs = [{"role": "user", "content": "first"}, {"role": "assistant", "content": "second"},
            {"role": "user", "content": [{"type": "text", "text": "multi"}, {"type": "text", "text": "part"}]},
            {"role": "assistant", "content": "fourth"}]
    for i, m in enumerate(msgs):  # all in the same second: only insertion order distinguishes them
        c.execute("INSERT INTO messages(id, thread_id, message, metadata, created_at) VALUES (?,?,?,?,?)",
                  (f"z{9 - i}", "t1", json.dumps(m), "{}", "2025-01-01 10:00:05"))
    c.commit()
    c.close()

    async def go():
        db = LocalDBClient(str(path))
        await db.initialize()
        got = await db.get_thread_messages("t1")
        assert [m.content for m in got] == ["first", "second", "multi\npart", "fourth"]
        from kafka_llm_service_amd.llm.types import Message
        await db.add_message("t1", Message(role="user", content="fifth"))
        assert (await db.get_thread_messages("t1"))[-1].content == "fifth"
        await db.close()
    asyncio.run(go())


def test_tokenizer_compression_on_reference_prompt():
    """Workload fidelity of the shipped BPE: trained on local text that is not the reference's
    prompt (scripts/build_tokenizer.py), it must compress the held-out reference sections like a Llama-3-class
    tokenizer (>= 3.8 chars/token; Llama-3 ~4.3) and render the served shared prefix — the reference's 13-section
    system prompt (/root/reference/src/prompts/v1.py:73-117) + the server's tool schemas — in <= 19k tokens
    (~18k)."""
    import asyncio
    from pathlib import Path

    from kafka_llm_service_amd.kafka.v1 import KafkaV1Provider
    from kafka_llm_service_amd.llm.stub import StubEchoProvider
    from kafka_llm_service_amd.sandbox.local import LocalSandbox
    from kafka_llm_service_amd.server_tools import NotebookTools, PlannerTools, ShellTools

    assert TOK.n_base == 128000 and TOK.vocab_size == 128256
    root = Path(__file__).resolve().parents[1] / "kafka_llm_service_amd/prompts/sections_reference"
    chars = toks = 0
    for f in sorted(root.rglob("*.md")):
        t = f.read_text(encoding="utf-8")
        chars += len(t)
        toks += len(TOK.encode(t))
        assert TOK.decode(TOK.encode(t)) == t
    assert chars / toks >= 3.8, chars / toks

    async def prefix():
        sb = LocalSandbox("http://127.0.0.1:9")
        kafka = KafkaV1Provider(StubEchoProvider(), tools=[get_weather_tool, count_tool] + PlannerTools(None).tools,
                                sandbox_tools=ShellTools(sb).tools + NotebookTools(sb).tools, mcp_servers=[])
        await kafka.initialize()
        return kafka.system_prompt, await kafka.get_tools()

    system, tools = asyncio.run(prefix())
    assert len(system) == 70496  # the reference's rendered default prompt, byte for byte
    ids = TPL.render([Message(role="system", content=system)], tools, add_generation_prompt=False)
    assert 15000 <= len(ids) <= 19000, len(ids)
