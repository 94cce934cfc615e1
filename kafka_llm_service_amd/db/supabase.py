"""Supabase (PostgREST) thread store — the optional hosted backend of the reference
(/root/reference/src/db/supabase.py:41-707), spoken directly over HTTP with httpx (the ``supabase`` SDK is not
installed; its sync client also blocked the event loop).

Same interface as ``LocalDBClient`` (the server picks it with ``KAFKA_DB=supabase`` + ``SUPABASE_URL`` /
``SUPABASE_KEY``). Schema, as the reference uses it:
  threads(id, user_id, kafka_profile_id, vm_api_key_id, sandbox_id, metadata, created_at)
  oai_messages(id, thread_id, message jsonb, metadata jsonb, created_at)   -- OpenAI message JSON in ``message``
  kafka_profiles(id, user_id, memory_dsn, global_prompt), profiles(id, <provider>_pk_virtual_key ...),
  vm_api_keys(id, api_key, user_id, status), playbooks(id, kafka_profile_id, name, description, created_at),
  rpc generate_vm_api_key() -> text.
Differences from the reference: history is ordered by ``created_at`` then ``id`` (the reference's same-second ties
came back in arbitrary order, quirk Q10 — deployments that can add a ``seq`` column set ``order_column="seq"``),
generated token ids ride inside the message JSON as ``kafka_token_ids`` (the thread token cache that keeps the KV
prefix hot), and nothing blocks the event loop.
"""
from __future__ import annotations

import asyncio
import json
import os
import secrets
import uuid
from collections import defaultdict
from datetime import datetime, timezone
from typing import Any

import httpx

from kafka_llm_service_amd.llm.types import Message

PROVIDER_KEYS = ("openai_pk_virtual_key", "anthropic_pk_virtual_key", "gemini_pk_virtual_key",
                 "bedrock_pk_virtual_key")


def _now() -> str:
    return datetime.now(timezone.utc).isoformat()


class SupabaseDBClient:
    def __init__(self, url: str | None = None, key: str | None = None, messages_table: str = "oai_messages",
                 threads_table: str = "threads", order_column: str = "created_at", transport=None):
        self.url = (url or os.environ.get("SUPABASE_URL", "")).rstrip("/")
        self.key = key or os.environ.get("SUPABASE_KEY", "")
        if not self.url:
            raise ValueError("SUPABASE_URL is not set")
        self.messages_table, self.threads_table = messages_table, threads_table
        self.order_column = order_column
        self._transport = transport
        self._client: httpx.AsyncClient | None = None
        self._locks: dict[str, asyncio.Lock] = defaultdict(asyncio.Lock)

    # --- plumbing ---------------------------------------------------------------------------------------------
    async def initialize(self) -> None:
        if self._client is None:
            self._client = httpx.AsyncClient(
                base_url=f"{self.url}/rest/v1", transport=self._transport, timeout=30.0,
                headers={"apikey": self.key, "Authorization": f"Bearer {self.key}",
                         "Content-Type": "application/json"})

    async def close(self) -> None:
        if self._client is not None:
            await self._client.aclose()
            self._client = None

    def thread_lock(self, thread_id: str) -> asyncio.Lock:
        return self._locks[thread_id]

    async def _req(self, method: str, path: str, params: dict | None = None, body: Any = None,
                   prefer: str | None = None) -> Any:
        await self.initialize()
        headers = {"Prefer": prefer} if prefer else None
        r = await self._client.request(method, path, params=params, json=body, headers=headers)
        if r.status_code >= 400:
            raise RuntimeError(f"PostgREST {method} {path} failed: {r.status_code} {r.text[:300]}")
        return r.json() if r.content else None

    # --- threads ----------------------------------------------------------------------------------------------
    async def create_thread(self, thread_id: str | None = None, system_message: str | None = None,
                            user_id: str | None = None, kafka_profile_id: str | None = None,
                            metadata: dict | None = None) -> dict[str, Any]:
        tid = thread_id or str(uuid.uuid4())
        row = {"id": tid, "metadata": metadata or {}, "created_at": _now()}
        if user_id:
            row["user_id"] = user_id
        if kafka_profile_id:
            row["kafka_profile_id"] = kafka_profile_id
        out = await self._req("POST", f"/{self.threads_table}", body=row,
                              prefer="return=representation,resolution=ignore-duplicates")
        created = (out[0] if out else row)["created_at"]
        if system_message:
            await self.add_message(tid, Message(role="system", content=system_message))
        return {"id": tid, "thread_id": tid, "created_at": created}

    async def thread_exists(self, thread_id: str) -> bool:
        rows = await self._req("GET", f"/{self.threads_table}", {"select": "id", "id": f"eq.{thread_id}"})
        return bool(rows)

    async def get_thread_metadata(self, thread_id: str) -> dict[str, Any] | None:
        rows = await self._req("GET", f"/{self.threads_table}", {"select": "*", "id": f"eq.{thread_id}"})
        return rows[0] if rows else None

    # --- messages ---------------------------------------------------------------------------------------------
    async def get_thread_messages(self, thread_id: str, limit: int | None = None,
                                  include_system: bool = True) -> list[Message]:
        params = {"select": "*", "thread_id": f"eq.{thread_id}", "order": f"{self.order_column}.asc,id.asc"}
        if limit:
            params["limit"] = str(limit)
        out = []
        for row in await self._req("GET", f"/{self.messages_table}", params) or []:
            d = row.get("message", row)
            if isinstance(d, str):
                d = json.loads(d)
            content = d.get("content")
            if isinstance(content, list):  # OpenAI multi-part content -> text (as the reference)
                content = "\n".join(p["text"] if isinstance(p, dict) else str(p) for p in content
                                    if isinstance(p, str) or (isinstance(p, dict) and "text" in p)) or None
            if not include_system and d.get("role") == "system":
                continue
            out.append(Message(role=d.get("role", "user"), content=content, name=d.get("name"),
                               tool_calls=d.get("tool_calls"), tool_call_id=d.get("tool_call_id"),
                               token_ids=d.get("kafka_token_ids")))
        return out

    def _row(self, thread_id: str, m: Message, metadata: dict | None) -> dict:
        d = m.to_dict()
        if m.token_ids:
            d["kafka_token_ids"] = list(m.token_ids)
        return {"id": str(uuid.uuid4()), "thread_id": thread_id, "message": d, "metadata": metadata or {},
                "created_at": _now()}

    async def _ensure_thread(self, thread_id: str) -> None:
        await self._req("POST", f"/{self.threads_table}", body={"id": thread_id, "metadata": {}, "created_at": _now()},
                        prefer="resolution=ignore-duplicates")

    async def add_message(self, thread_id: str, message: Message, metadata: dict | None = None) -> str:
        return (await self.add_messages(thread_id, [message], metadata))[0]

    async def add_messages(self, thread_id: str, messages: list[Message], metadata: dict | None = None) -> list[str]:
        await self._ensure_thread(thread_id)
        rows = [self._row(thread_id, m, metadata) for m in messages]
        await self._req("POST", f"/{self.messages_table}", body=rows, prefer="return=minimal")
        return [r["id"] for r in rows]

    async def delete_thread_messages(self, thread_id: str) -> int:
        rows = await self._req("DELETE", f"/{self.messages_table}", {"thread_id": f"eq.{thread_id}"},
                               prefer="return=representation")
        return len(rows or [])

    # --- sandbox / config -------------------------------------------------------------------------------------
    async def get_thread_sandbox_id(self, thread_id: str) -> str | None:
        rows = await self._req("GET", f"/{self.threads_table}", {"select": "sandbox_id", "id": f"eq.{thread_id}"})
        return rows[0].get("sandbox_id") if rows else None

    async def update_thread_sandbox_id(self, thread_id: str, sandbox_id: str | None) -> bool:
        rows = await self._req("PATCH", f"/{self.threads_table}", {"id": f"eq.{thread_id}"},
                               body={"sandbox_id": sandbox_id}, prefer="return=representation")
        return bool(rows)

    async def get_thread_config(self, thread_id: str) -> dict[str, Any] | None:
        """Thread -> kafka_profiles (memory_dsn, global_prompt) -> profiles (provider virtual keys), vm_api_keys."""
        rows = await self._req("GET", f"/{self.threads_table}", {
            "select": "id,user_id,kafka_profile_id,vm_api_key_id", "id": f"eq.{thread_id}"})
        if not rows:
            return None
        t = rows[0]
        kp = {}
        if t.get("kafka_profile_id"):
            r = await self._req("GET", "/kafka_profiles", {"select": "user_id,memory_dsn,global_prompt",
                                                           "id": f"eq.{t['kafka_profile_id']}"})
            kp = r[0] if r else {}
        keys = {k: None for k in PROVIDER_KEYS}
        if kp.get("user_id"):
            r = await self._req("GET", "/profiles", {"select": ",".join(PROVIDER_KEYS), "id": f"eq.{kp['user_id']}"})
            if r:
                keys.update({k: r[0].get(k) for k in PROVIDER_KEYS})
        vm = None
        if t.get("vm_api_key_id"):
            r = await self._req("GET", "/vm_api_keys", {"select": "api_key", "id": f"eq.{t['vm_api_key_id']}"})
            vm = r[0]["api_key"] if r else None
        return {"thread_id": t["id"], "user_id": t.get("user_id"), "kafka_profile_id": t.get("kafka_profile_id"),
                "memory_dsn": kp.get("memory_dsn"), "global_prompt": kp.get("global_prompt"), **keys,
                "virtual_keys": {k: v for k, v in keys.items() if v}, "vm_api_key": vm}

    async def get_playbooks_for_kafka_profile(self, kafka_profile_id: str) -> list[dict[str, Any]]:
        return await self._req("GET", "/playbooks", {"select": "id,name,description,created_at",
                                                     "kafka_profile_id": f"eq.{kafka_profile_id}",
                                                     "order": "created_at.asc,id.asc"}) or []

    async def get_or_create_vm_api_key(self, thread_id: str, user_id: str | None = None) -> str:
        """The thread's active VM key; else a new one from the ``generate_vm_api_key`` RPC (falling back to a local
        random key if the RPC is unavailable, as the reference does, supabase.py:584-587), linked to the thread."""
        rows = await self._req("GET", f"/{self.threads_table}", {"select": "vm_api_key_id", "id": f"eq.{thread_id}"})
        kid = rows[0].get("vm_api_key_id") if rows else None
        if kid:
            r = await self._req("GET", "/vm_api_keys", {"select": "api_key,status", "id": f"eq.{kid}"})
            if r and r[0].get("status", "active") == "active":
                return r[0]["api_key"]
        try:
            key = await self._req("POST", "/rpc/generate_vm_api_key", body={})
        except RuntimeError:
            key = None
        if not isinstance(key, str) or not key:
            key = "vmk_" + secrets.token_hex(24)
        kid = str(uuid.uuid4())
        await self._req("POST", "/vm_api_keys", body={"id": kid, "api_key": key, "user_id": user_id,
                                                      "status": "active"}, prefer="return=minimal")
        await self._req("PATCH", f"/{self.threads_table}", {"id": f"eq.{thread_id}"}, body={"vm_api_key_id": kid})
        return key
