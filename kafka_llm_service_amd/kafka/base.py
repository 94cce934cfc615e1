"""KafkaAgent: thread-aware wrapper around the agent loop (/root/reference/src/kafka/base.py:24-319).

``run_with_thread``: ensure the thread exists, load its history (seq-ordered), sanitise orphan tool messages, persist
the new user/system messages BEFORE the run, stream the agent events, and persist every assistant turn (with its
engine token ids) and tool result as they complete. The whole read-run-persist sequence holds the thread's lock, so
two concurrent requests on one thread cannot interleave their history (quirk Q11).
"""
from __future__ import annotations

import contextlib
from abc import ABC, abstractmethod
from typing import Any, AsyncGenerator

from kafka_llm_service_amd.kafka.utils import sanitize_messages_for_openai
from kafka_llm_service_amd.llm.types import Message
from kafka_llm_service_amd.obs import trace


class KafkaAgent(ABC):
    def __init__(self, thread_id: str | None = None, db_client=None):
        self._thread_id = thread_id
        self._db_client = db_client

    @property
    def thread_id(self) -> str | None:
        return self._thread_id

    @abstractmethod
    async def initialize(self) -> None: ...

    @abstractmethod
    async def cleanup(self) -> None: ...

    @abstractmethod
    async def get_tools(self) -> list[dict[str, Any]]: ...

    @abstractmethod
    def run(self, messages: list[Message], model: str, temperature: float = 0.7, max_tokens: int | None = None,
            **kwargs) -> AsyncGenerator[dict[str, Any], None]: ...

    async def ensure_thread_exists(self) -> None:
        if self._thread_id and self._db_client and not await self._db_client.thread_exists(self._thread_id):
            await self._db_client.create_thread(thread_id=self._thread_id)

    async def get_thread_messages(self) -> list[Message]:
        if not self._thread_id or not self._db_client:
            return []
        return await self._db_client.get_thread_messages(self._thread_id)

    async def save_message(self, message: Message) -> None:
        if self._thread_id and self._db_client:
            await self._db_client.add_message(self._thread_id, message)

    async def save_messages(self, messages: list[Message]) -> None:
        if self._thread_id and self._db_client and messages:
            await self._db_client.add_messages(self._thread_id, messages)

    async def run_with_thread(self, new_messages: list[Message], model: str, temperature: float = 0.7,
                              max_tokens: int | None = None, save_to_thread: bool = True, thread_id: str | None = None,
                              db_client=None, **kwargs) -> AsyncGenerator[dict[str, Any], None]:
        """``thread_id`` / ``db_client`` override the bound ones, so one (global) agent can serve many threads."""
        tid = thread_id or self._thread_id
        db = db_client or self._db_client
        lock = db.thread_lock(tid) if (tid and db is not None and hasattr(db, "thread_lock")) else _async_null()
        async with lock:
            history: list[Message] = []
            with trace.span("api_db_load", "api", f"thr:{tid}"):
                if tid and db is not None:
                    if not await db.thread_exists(tid):
                        await db.create_thread(thread_id=tid)
                    history = await db.get_thread_messages(tid)
                msgs = sanitize_messages_for_openai(history + list(new_messages))
            behind = hasattr(db, "sync")  # a store with write-behind: saves leave the time-to-first-token path
            if save_to_thread and tid and db is not None:
                new = [m for m in new_messages if m.role in ("user", "system")]
                if new:
                    with trace.span("api_db_save", "api", f"thr:{tid}"):
                        if behind:
                            await db.add_messages(tid, new, wait=False)
                        else:
                            await db.add_messages(tid, new)
            try:
                async for ev in self.run(msgs, model=model, temperature=temperature, max_tokens=max_tokens,
                                         emit_messages=True, **kwargs):
                    if ev.get("type") == "_message":
                        if save_to_thread and tid and db is not None:
                            if behind:
                                await db.add_message(tid, ev["message"], wait=False)
                            else:
                                await db.add_message(tid, ev["message"])
                        continue
                    yield ev
            finally:
                if behind:
                    await db.sync()  # every write of this request is in SQLite before the thread lock is released

    async def __aenter__(self) -> "KafkaAgent":
        await self.initialize()
        return self

    async def __aexit__(self, *exc) -> None:
        await self.cleanup()


@contextlib.asynccontextmanager
async def _async_null():
    yield
