"""The Supabase (PostgREST) thread store against an in-process fake PostgREST (eq filters, select, order, limit,
upsert-ignore, PATCH/DELETE with representation, RPC) — same behaviour as the SQLite store, plus the reference's
thread-config join."""
import asyncio
import json

import httpx
import pytest

from kafka_llm_service_amd.db.supabase import SupabaseDBClient
from kafka_llm_service_amd.llm.types import Message


class FakePostgREST:
    def __init__(self):
        self.tables: dict[str, list[dict]] = {}

    def _match(self, row, params):
        for k, v in params.items():
            if k in ("select", "order", "limit"):
                continue
            op, _, val = v.partition(".")
            if op == "eq" and str(row.get(k)) != val:
                return False
        return True

    def handler(self, req: httpx.Request) -> httpx.Response:
        path = req.url.path.split("/rest/v1/")[1]
        params = dict(req.url.params)
        if path.startswith("rpc/"):
            return httpx.Response(200, json="vmk_from_rpc")
        rows = self.tables.setdefault(path, [])
        prefer = req.headers.get("prefer", "")
        if req.method == "GET":
            out = [r for r in rows if self._match(r, params)]
            if "order" in params:
                for key in reversed(params["order"].split(",")):
                    col, _, d = key.partition(".")
                    out.sort(key=lambda r: str(r.get(col)), reverse=(d == "desc"))
            if "limit" in params:
                out = out[:int(params["limit"])]
            if params.get("select", "*") != "*":
                cols = params["select"].split(",")
                out = [{c: r.get(c) for c in cols} for r in out]
            return httpx.Response(200, json=out)
        if req.method == "POST":
            body = json.loads(req.content)
            new = body if isinstance(body, list) else [body]
            added = []
            for r in new:
                if "ignore-duplicates" in prefer and any(x.get("id") == r.get("id") for x in rows):
                    continue
                rows.append(dict(r))
                added.append(r)
            return httpx.Response(201, json=added if "representation" in prefer else None)
        if req.method == "PATCH":
            body = json.loads(req.content)
            hit = [r for r in rows if self._match(r, params)]
            for r in hit:
                r.update(body)
            return httpx.Response(200, json=hit if "representation" in prefer else None)
        if req.method == "DELETE":
            hit = [r for r in rows if self._match(r, params)]
            self.tables[path] = [r for r in rows if r not in hit]
            return httpx.Response(200, json=hit)
        return httpx.Response(405)


@pytest.fixture()
def db():
    fake = FakePostgREST()
    c = SupabaseDBClient(url="http://supabase.test", key="k", transport=httpx.MockTransport(fake.handler))
    c.fake = fake
    return c


def test_thread_and_message_roundtrip(db):
    async def go():
        t = await db.create_thread(system_message="be brief", user_id="u1")
        tid = t["id"]
        assert await db.thread_exists(tid) and not await db.thread_exists("nope")
        await db.add_messages(tid, [Message(role="user", content="hi"),
                                    Message(role="assistant", content="yo", token_ids=[1, 2, 3])])
        msgs = await db.get_thread_messages(tid)
        assert [m.role for m in msgs] == ["system", "user", "assistant"] and msgs[2].token_ids == [1, 2, 3]
        assert [m.role for m in await db.get_thread_messages(tid, include_system=False)] == ["user", "assistant"]
        assert await db.update_thread_sandbox_id(tid, "sb-1") and await db.get_thread_sandbox_id(tid) == "sb-1"
        assert await db.delete_thread_messages(tid) == 3 and await db.get_thread_messages(tid) == []
        # auto-created thread on add_message
        await db.add_message("auto-1", Message(role="user", content="x"))
        assert await db.thread_exists("auto-1")
        await db.close()
    asyncio.run(go())


def test_thread_config_join_playbooks_and_vm_key(db):
    f = db.fake
    f.tables["kafka_profiles"] = [{"id": "kp1", "user_id": "owner", "memory_dsn": "pg://m", "global_prompt": "GP"}]
    f.tables["profiles"] = [{"id": "owner", "openai_pk_virtual_key": "vk-oa"}]
    f.tables["playbooks"] = [{"id": "b", "kafka_profile_id": "kp1", "name": "N2", "description": "D2",
                              "created_at": "2"},
                             {"id": "a", "kafka_profile_id": "kp1", "name": "N1", "description": "D1",
                              "created_at": "1"}]

    async def go():
        await db.create_thread(thread_id="t1", kafka_profile_id="kp1")
        cfg = await db.get_thread_config("t1")
        assert cfg["global_prompt"] == "GP" and cfg["memory_dsn"] == "pg://m"
        assert cfg["openai_pk_virtual_key"] == "vk-oa" and cfg["virtual_keys"] == {"openai_pk_virtual_key": "vk-oa"}
        assert [p["name"] for p in await db.get_playbooks_for_kafka_profile("kp1")] == ["N1", "N2"]
        k1 = await db.get_or_create_vm_api_key("t1", "owner")
        assert k1 == "vmk_from_rpc" and await db.get_or_create_vm_api_key("t1") == k1
        assert (await db.get_thread_config("t1"))["vm_api_key"] == k1
        await db.close()
    asyncio.run(go())


def test_local_db_cache_and_write_behind(tmp_path):
    """The history cache answers reads without SQLite, write-behind saves keep their order (seq) and are durable
    after sync(), and a fresh client on the same file sees exactly what the cached one served."""
    import asyncio

    from kafka_llm_service_amd.db.local import LocalDBClient
    from kafka_llm_service_amd.llm.types import Message

    async def main():
        path = str(tmp_path / "t.db")
        db = LocalDBClient(path)
        await db.initialize()
        await db.create_thread(thread_id="t1", system_message="sys")
        assert [m.content for m in await db.get_thread_messages("t1")] == ["sys"]  # now cached
        for i in range(20):
            await db.add_messages("t1", [Message(role="user", content=f"u{i}")], wait=False)
            await db.add_message("t1", Message(role="assistant", content=f"a{i}", token_ids=[i, i + 1]), wait=False)
        got = await db.get_thread_messages("t1")
        assert [m.content for m in got][:3] == ["sys", "u0", "a0"] and len(got) == 41
        got[1].content = "edited by a caller"  # must not leak into the cache
        assert (await db.get_thread_messages("t1"))[1].content == "u0"
        await db.sync()
        fresh = LocalDBClient(path)
        await fresh.initialize()
        back = await fresh.get_thread_messages("t1")
        assert [m.content for m in back] == [m.content for m in await db.get_thread_messages("t1")]
        assert back[2].token_ids == [0, 1]
        assert await db.delete_thread_messages("t1") == 41 and await db.get_thread_messages("t1") == []
        await db.close()
        await fresh.close()

    asyncio.run(main())


def test_local_db_failed_write_behind_is_reported(tmp_path):
    """A write-behind save that fails is raised by sync() and its thread leaves the history cache, so the store
    never keeps serving rows SQLite does not have (the error used to be swallowed by the callback)."""
    import asyncio

    import pytest

    from kafka_llm_service_amd.db.local import LocalDBClient
    from kafka_llm_service_amd.llm.types import Message

    async def main():
        db = LocalDBClient(str(tmp_path / "f.db"))
        await db.initialize()
        await db.create_thread(thread_id="t1", system_message="sys")
        assert len(await db.get_thread_messages("t1")) == 1  # cached
        real = db._insert
        calls = {"n": 0}

        def flaky(c, tid, m, meta, mid):
            calls["n"] += 1
            if m.content == "boom":
                raise RuntimeError("disk full")
            return real(c, tid, m, meta, mid)

        db._insert = flaky
        await db.add_messages("t1", [Message(role="user", content="ok"), Message(role="user", content="boom")],
                              wait=False)
        with pytest.raises(RuntimeError, match="disk full"):
            await db.sync()
        await db.sync()  # reported once
        db._insert = real
        # the whole failed call rolled back; the cache was dropped, so the read comes from SQLite
        assert [m.content for m in await db.get_thread_messages("t1")] == ["sys"]
        await db.close()

    asyncio.run(main())


def test_local_db_cache_miss_race_does_not_cache_stale_history(tmp_path):
    """A history read that misses the cache and races a write queued after it must not cache what it read: the
    per-thread write generation (bumped by add_messages / delete_thread_messages) makes the fill a no-op."""
    import asyncio

    from kafka_llm_service_amd.db.local import LocalDBClient
    from kafka_llm_service_amd.llm.types import Message

    async def main():
        db = LocalDBClient(str(tmp_path / "r.db"))
        await db.initialize()
        await db.create_thread(thread_id="t1", system_message="sys")
        db._cache.clear()
        read = asyncio.ensure_future(db.get_thread_messages("t1"))  # queued first: sees only "sys"
        await asyncio.sleep(0)
        await db.add_message("t1", Message(role="user", content="new"))  # wait=True, queued after the read
        assert [m.content for m in await read] == ["sys"]
        assert "t1" not in db._cache  # the stale read was not cached
        assert [m.content for m in await db.get_thread_messages("t1")] == ["sys", "new"]
        await db.close()

    asyncio.run(main())


def test_local_db_new_thread_history_is_cached_at_creation(tmp_path):
    """A thread created by this client starts with its (empty) history cached, so the first turn's history load
    never queues behind other threads' SQLite I/O (HTTP burst TTFT); re-creating an EXISTING thread (INSERT OR
    IGNORE) must not cache an empty history over its stored rows."""
    import asyncio

    from kafka_llm_service_amd.db.local import LocalDBClient
    from kafka_llm_service_amd.llm.types import Message

    async def main():
        path = str(tmp_path / "c.db")
        db = LocalDBClient(path)
        await db.initialize()
        await db.create_thread(thread_id="t1")
        await db.add_message("t1", Message(role="user", content="hi"))
        real = db._connect
        db._connect = lambda: (_ for _ in ()).throw(AssertionError("history read went to SQLite"))
        assert [m.content for m in await db.get_thread_messages("t1")] == ["hi"]
        db._connect = real
        await db.close()
        other = LocalDBClient(path)
        await other.initialize()
        await other.create_thread(thread_id="t1")  # already exists: nothing cached
        assert "t1" not in other._cache
        assert [m.content for m in await other.get_thread_messages("t1")] == ["hi"]
        await other.close()

    asyncio.run(main())
