"""Thread / message store on SQLite — the source of truth for conversation state.

Interface parity with /root/reference/src/db/local.py:20-370 and the Supabase client's thread-config surface
(/root/reference/src/db/supabase.py:458-707): get_thread_messages / add_message(s) / create_thread / thread_exists /
get_thread_metadata / delete_thread_messages / get|update_thread_sandbox_id / get_thread_config /
get_or_create_vm_api_key / get_playbooks_for_kafka_profile.

Fixed vs the reference:
  * ordering is a monotonic per-thread ``seq`` (the reference ordered by ``created_at`` with 1-second resolution, so
    same-second messages could come back in any order — quirk Q10); a database written by the reference is migrated
    in place on open (columns added, ``seq`` assigned in created_at / insertion order),
  * ``thread_lock(thread_id)`` serialises read-modify-write of one thread across concurrent requests (Q11),
  * every message row keeps the engine token ids of generated assistant turns (``token_ids`` column): the chat
    template re-renders history from them exactly, which keeps the thread's KV prefix cache hot,
  * all SQLite work runs on one dedicated thread (sqlite3 connections are not thread-safe; aiosqlite is not
    installed) so the API event loop never blocks on disk I/O (the reference's Supabase client blocked the loop),
  * a write-through cache of recent threads' histories (``LOCAL_DB_CACHE_THREADS``, default 4096; 0 = off) serves
    the per-request history read without a trip through the SQLite thread, and ``add_messages(wait=False)`` queues
    a write behind the ones before it (one FIFO writer: order and ``seq`` are kept) so the new user message's save
    is off the time-to-first-token path; ``sync()`` waits for every queued write (the agent calls it before a
    request ends). The cache assumes this process is the database's only writer (one server process per file).
"""
from __future__ import annotations

import asyncio
import json
import os
import secrets
import sqlite3
import uuid
from collections import OrderedDict, defaultdict
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from typing import Any

from kafka_llm_service_amd.llm.types import Message

SCHEMA = """
CREATE TABLE IF NOT EXISTS threads (
    id TEXT PRIMARY KEY, created_at TEXT NOT NULL, metadata TEXT, sandbox_id TEXT, user_id TEXT,
    kafka_profile_id TEXT, next_seq INTEGER NOT NULL DEFAULT 0);
CREATE TABLE IF NOT EXISTS messages (
    id TEXT PRIMARY KEY, thread_id TEXT NOT NULL REFERENCES threads(id), seq INTEGER NOT NULL,
    message TEXT NOT NULL, token_ids TEXT, metadata TEXT, created_at TEXT NOT NULL);
CREATE TABLE IF NOT EXISTS kafka_profiles (
    id TEXT PRIMARY KEY, user_id TEXT, global_prompt TEXT, memory_dsn TEXT, virtual_keys TEXT);
CREATE TABLE IF NOT EXISTS playbooks (
    id TEXT PRIMARY KEY, kafka_profile_id TEXT, name TEXT, description TEXT, created_at TEXT);
CREATE TABLE IF NOT EXISTS vm_api_keys (
    id TEXT PRIMARY KEY, thread_id TEXT, user_id TEXT, api_key TEXT, status TEXT, created_at TEXT);
"""


INDEXES = """
CREATE UNIQUE INDEX IF NOT EXISTS idx_messages_thread_seq ON messages(thread_id, seq);
"""


def _migrate(c: sqlite3.Connection) -> None:
    """Open a database written by the reference service (/root/reference/src/db/local.py:51-76: threads(id,
    created_at, metadata, sandbox_id), messages(id, thread_id, message, metadata, created_at), ordered by the
    1-second ``created_at``): add the columns this store uses and give existing messages a ``seq`` in their original
    order (created_at, then insertion order), so a user can switch over with their thread history intact."""
    tcols = {r[1] for r in c.execute("PRAGMA table_info(threads)")}
    for col, decl in (("user_id", "TEXT"), ("kafka_profile_id", "TEXT"),
                      ("next_seq", "INTEGER NOT NULL DEFAULT 0"), ("sandbox_id", "TEXT"), ("metadata", "TEXT")):
        if col not in tcols:
            c.execute(f"ALTER TABLE threads ADD COLUMN {col} {decl}")
    mcols = {r[1] for r in c.execute("PRAGMA table_info(messages)")}
    if "token_ids" not in mcols:
        c.execute("ALTER TABLE messages ADD COLUMN token_ids TEXT")
    if "seq" not in mcols:
        c.execute("ALTER TABLE messages ADD COLUMN seq INTEGER")
        rows = c.execute("SELECT rowid, thread_id FROM messages ORDER BY thread_id, created_at, rowid").fetchall()
        counts: dict[str, int] = {}
        for rowid, tid in rows:
            n = counts.get(tid, 0)
            c.execute("UPDATE messages SET seq=? WHERE rowid=?", (n, rowid))
            counts[tid] = n + 1
        for tid, n in counts.items():
            c.execute("INSERT OR IGNORE INTO threads(id, created_at, metadata) VALUES (?,?,?)", (tid, _now(), "{}"))
            c.execute("UPDATE threads SET next_seq=? WHERE id=?", (n, tid))
    c.commit()


def _flatten_content(d: dict) -> dict:
    """OpenAI multi-part content ([{"type": "text", "text": ...}, ...]) -> newline-joined text, as the reference
    does on read (/root/reference/src/db/local.py:123-132); Message.content is a string."""
    c = d.get("content")
    if isinstance(c, list):
        parts = [p["text"] if isinstance(p, dict) else str(p) for p in c
                 if isinstance(p, str) or (isinstance(p, dict) and "text" in p)]
        d["content"] = "\n".join(parts) if parts else None
    return d


def _now() -> str:
    return datetime.now(timezone.utc).isoformat()


class LocalDBClient:
    def __init__(self, db_path: str | None = None):
        self.db_path = db_path or os.environ.get("LOCAL_DB_PATH", "data/threads.db")
        self._exec = ThreadPoolExecutor(max_workers=1, thread_name_prefix="kafka-sqlite")
        self._conn: sqlite3.Connection | None = None
        self._locks: dict[str, asyncio.Lock] = defaultdict(asyncio.Lock)
        self._initialized = False
        self._cache_n = int(os.environ.get("LOCAL_DB_CACHE_THREADS", "4096"))
        self._cache: OrderedDict[str, list[Message]] = OrderedDict()  # thread id -> full history, seq order
        self._known: set[str] = set()
        self._pending: set = set()  # write-behind futures not yet awaited
        self._write_error: BaseException | None = None  # first failed write-behind save, raised by sync()
        self._gen: dict[str, int] = defaultdict(int)  # per-thread write generation (guards cache fills on a miss)

    # --- plumbing ---------------------------------------------------------------------------------------------
    def _connect(self) -> sqlite3.Connection:
        if self._conn is None:
            if self.db_path != ":memory:":
                os.makedirs(os.path.dirname(os.path.abspath(self.db_path)), exist_ok=True)
            self._conn = sqlite3.connect(self.db_path, check_same_thread=False)
            self._conn.row_factory = sqlite3.Row
            self._conn.execute("PRAGMA journal_mode=WAL")
            self._conn.execute("PRAGMA synchronous=NORMAL")
            self._conn.executescript(SCHEMA)
            _migrate(self._conn)
            self._conn.executescript(INDEXES)
        return self._conn

    async def _run(self, fn, *args):
        return await asyncio.get_running_loop().run_in_executor(self._exec, fn, *args)

    def _cache_put(self, thread_id: str, msgs: list[Message]) -> None:
        if self._cache_n <= 0:
            return
        self._cache[thread_id] = msgs
        self._cache.move_to_end(thread_id)
        while len(self._cache) > self._cache_n:
            self._cache.popitem(last=False)

    async def sync(self) -> None:
        """Wait until every queued write has reached SQLite (the writer is FIFO: a no-op behind them suffices) and
        raise the first write-behind failure since the last sync (its thread was dropped from the cache, so the
        history served afterwards is what SQLite holds)."""
        if self._pending:
            await self._run(lambda: None)
            for f in list(self._pending):
                if f.done():
                    self._pending.discard(f)
        err, self._write_error = self._write_error, None
        if err is not None:
            raise err

    def _write_failed(self, thread_id: str, fut) -> None:
        """Done-callback of a write-behind save: on failure keep the error for sync() and forget the thread's cached
        history (it already shows the rows that did not reach SQLite)."""
        self._pending.discard(fut)
        exc = None if fut.cancelled() else fut.exception()
        if exc is not None:
            self._cache.pop(thread_id, None)
            self._gen[thread_id] += 1
            if self._write_error is None:
                self._write_error = exc

    async def initialize(self) -> None:
        await self._run(self._connect)
        self._initialized = True

    async def close(self) -> None:
        def _close():
            if self._conn is not None:
                self._conn.close()
                self._conn = None
        await self._run(_close)

    def thread_lock(self, thread_id: str) -> asyncio.Lock:
        """Per-thread lock: hold it across read-history -> run -> persist for one request."""
        return self._locks[thread_id]

    # --- threads ----------------------------------------------------------------------------------------------
    async def create_thread(self, thread_id: str | None = None, system_message: str | None = None,
                            user_id: str | None = None, kafka_profile_id: str | None = None,
                            metadata: dict | None = None) -> dict[str, Any]:
        tid = thread_id or str(uuid.uuid4())
        created = _now()

        def _do():
            c = self._connect()
            cur = c.execute("INSERT OR IGNORE INTO threads(id, created_at, metadata, user_id, kafka_profile_id) "
                            "VALUES (?,?,?,?,?)", (tid, created, json.dumps(metadata or {}), user_id, kafka_profile_id))
            c.commit()
            return cur.rowcount == 1
        gen = self._gen[tid]
        fresh = await self._run(_do)
        self._known.add(tid)
        if fresh and self._gen[tid] == gen and tid not in self._cache:
            # a thread created here has no rows: its (empty) history goes into the cache now, so the first turn's
            # history load is a cache hit instead of a SQLite read queued behind a burst of other threads' I/O on
            # the single writer thread (HTTP burst TTFT, VERDICT r02: api_db_load p99 93 ms)
            self._cache_put(tid, [])
        if system_message:
            await self.add_message(tid, Message(role="system", content=system_message))
        return {"id": tid, "thread_id": tid, "created_at": created}

    async def thread_exists(self, thread_id: str) -> bool:
        if thread_id in self._known:
            return True

        def _do():
            return self._connect().execute("SELECT 1 FROM threads WHERE id=?", (thread_id,)).fetchone() is not None
        ok = await self._run(_do)
        if ok:
            self._known.add(thread_id)
        return ok

    async def get_thread_metadata(self, thread_id: str) -> dict[str, Any] | None:
        def _do():
            r = self._connect().execute("SELECT * FROM threads WHERE id=?", (thread_id,)).fetchone()
            if r is None:
                return None
            d = dict(r)
            d["metadata"] = json.loads(d["metadata"] or "{}")
            return d
        return await self._run(_do)

    # --- messages ---------------------------------------------------------------------------------------------
    async def get_thread_messages(self, thread_id: str, limit: int | None = None,
                                  include_system: bool = True) -> list[Message]:
        hit = self._cache.get(thread_id)
        if hit is not None:
            self._cache.move_to_end(thread_id)
            out = [m.model_copy() for m in hit if include_system or m.role != "system"]  # callers may edit them
            return out[:limit] if limit else out

        gen = self._gen[thread_id]  # a write or delete queued after this read makes its result stale for the cache

        def _do():
            q = "SELECT message, token_ids FROM messages WHERE thread_id=? ORDER BY seq ASC"
            args: list[Any] = [thread_id]
            if limit:
                q += " LIMIT ?"
                args.append(limit)
            return self._connect().execute(q, args).fetchall()
        rows = await self._run(_do)
        out = []
        for r in rows:
            d = _flatten_content(json.loads(r["message"]))
            if not include_system and d.get("role") == "system":
                continue
            if r["token_ids"]:
                d["token_ids"] = json.loads(r["token_ids"])
            out.append(Message.from_dict(d))
        # (writes queued BEFORE the read are in it: one FIFO writer thread; later ones bumped the generation)
        if not limit and include_system and self._gen[thread_id] == gen:
            self._cache_put(thread_id, [m.model_copy() for m in out])
        return out

    def _insert(self, c: sqlite3.Connection, thread_id: str, m: Message, metadata: dict | None, mid: str) -> str:
        c.execute("INSERT OR IGNORE INTO threads(id, created_at, metadata) VALUES (?,?,?)",
                  (thread_id, _now(), "{}"))
        seq = c.execute("UPDATE threads SET next_seq = next_seq + 1 WHERE id=? RETURNING next_seq - 1",
                        (thread_id,)).fetchone()[0]
        c.execute("INSERT INTO messages(id, thread_id, seq, message, token_ids, metadata, created_at) "
                  "VALUES (?,?,?,?,?,?,?)",
                  (mid, thread_id, seq, json.dumps(m.to_dict()), json.dumps(m.token_ids) if m.token_ids else None,
                   json.dumps(metadata or {}), _now()))
        return mid

    async def add_message(self, thread_id: str, message: Message, metadata: dict | None = None,
                          wait: bool = True) -> str:
        return (await self.add_messages(thread_id, [message], metadata, wait))[0]

    async def add_messages(self, thread_id: str, messages: list[Message], metadata: dict | None = None,
                           wait: bool = True) -> list[str]:
        """Append in order. ``wait=False``: queue the write behind the earlier ones and return at once (the cache
        already shows the messages; ``sync()`` waits for the write)."""
        ids = [str(uuid.uuid4()) for _ in messages]
        msgs = list(messages)

        def _do():
            c = self._connect()
            try:
                for m, mid in zip(msgs, ids):
                    self._insert(c, thread_id, m, metadata, mid)
                c.commit()
            except BaseException:
                c.rollback()  # all of this call's rows or none
                raise
            return ids
        self._gen[thread_id] += 1
        hit = self._cache.get(thread_id)
        if hit is not None:
            hit.extend(m.model_copy() for m in msgs)
        self._known.add(thread_id)
        fut = asyncio.get_running_loop().run_in_executor(self._exec, _do)
        if wait:
            try:
                return await fut
            except BaseException:
                self._cache.pop(thread_id, None)  # the cache already showed the rows
                raise
        self._pending.add(fut)
        fut.add_done_callback(lambda f: self._write_failed(thread_id, f))
        return ids

    async def delete_thread_messages(self, thread_id: str) -> int:
        self._cache.pop(thread_id, None)
        self._gen[thread_id] += 1

        def _do():
            c = self._connect()
            n = c.execute("DELETE FROM messages WHERE thread_id=?", (thread_id,)).rowcount
            c.commit()
            return n
        return await self._run(_do)

    # --- sandbox / config -------------------------------------------------------------------------------------
    async def get_thread_sandbox_id(self, thread_id: str) -> str | None:
        meta = await self.get_thread_metadata(thread_id)
        return meta.get("sandbox_id") if meta else None

    async def update_thread_sandbox_id(self, thread_id: str, sandbox_id: str | None) -> bool:
        def _do():
            c = self._connect()
            n = c.execute("UPDATE threads SET sandbox_id=? WHERE id=?", (sandbox_id, thread_id)).rowcount
            c.commit()
            return n > 0
        return await self._run(_do)

    async def upsert_kafka_profile(self, profile_id: str, user_id: str | None = None, global_prompt: str | None = None,
                                   memory_dsn: str | None = None, virtual_keys: dict | None = None) -> None:
        def _do():
            c = self._connect()
            c.execute("INSERT OR REPLACE INTO kafka_profiles(id, user_id, global_prompt, memory_dsn, virtual_keys) "
                      "VALUES (?,?,?,?,?)", (profile_id, user_id, global_prompt, memory_dsn,
                                             json.dumps(virtual_keys or {})))
            c.commit()
        await self._run(_do)

    async def add_playbook(self, kafka_profile_id: str, name: str, description: str) -> str:
        pid = str(uuid.uuid4())

        def _do():
            c = self._connect()
            c.execute("INSERT INTO playbooks(id, kafka_profile_id, name, description, created_at) VALUES (?,?,?,?,?)",
                      (pid, kafka_profile_id, name, description, _now()))
            c.commit()
        await self._run(_do)
        return pid

    async def get_thread_config(self, thread_id: str) -> dict[str, Any] | None:
        """Thread -> kafka profile join: global_prompt, memory_dsn, virtual keys, user id (None if no profile)."""
        def _do():
            r = self._connect().execute(
                "SELECT t.user_id, t.kafka_profile_id, p.global_prompt, p.memory_dsn, p.virtual_keys "
                "FROM threads t LEFT JOIN kafka_profiles p ON p.id = t.kafka_profile_id WHERE t.id=?",
                (thread_id,)).fetchone()
            return dict(r) if r else None
        r = await self._run(_do)
        if r is None or not r.get("kafka_profile_id"):
            return None
        r["virtual_keys"] = json.loads(r.get("virtual_keys") or "{}")
        return r

    async def get_playbooks_for_kafka_profile(self, kafka_profile_id: str) -> list[dict[str, Any]]:
        def _do():
            return [dict(r) for r in self._connect().execute(
                "SELECT id, name, description, created_at FROM playbooks WHERE kafka_profile_id=? "
                "ORDER BY created_at, id", (kafka_profile_id,)).fetchall()]
        return await self._run(_do)

    async def get_or_create_vm_api_key(self, thread_id: str, user_id: str | None = None) -> str:
        def _do():
            c = self._connect()
            r = c.execute("SELECT api_key FROM vm_api_keys WHERE thread_id=? AND status='active'",
                          (thread_id,)).fetchone()
            if r:
                return r["api_key"]
            key = "vmk_" + secrets.token_hex(24)
            c.execute("INSERT INTO vm_api_keys(id, thread_id, user_id, api_key, status, created_at) "
                      "VALUES (?,?,?,?,?,?)", (str(uuid.uuid4()), thread_id, user_id, key, "active", _now()))
            c.commit()
            return key
        return await self._run(_do)


class MemoryDBClient(LocalDBClient):
    """Same store on an in-memory SQLite database (tests, benchmarks, stateless deployments)."""

    def __init__(self):
        super().__init__(db_path=":memory:")
