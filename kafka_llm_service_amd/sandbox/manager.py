"""Per-thread sandbox lifecycle (/root/reference/src/sandbox/manager.py:37-458) over a pluggable provisioner.

* ``get_sandbox_if_ready(thread_id)`` — non-blocking: cached + healthy (claim if unclaimed), else the thread's
  recorded sandbox id re-connected through the provisioner, else None (stale cache entries are evicted);
* ``ensure_sandbox_background(thread_id)`` — fire-and-forget create/claim task (one per thread, tracked so
  concurrent requests do not start two); ``is_sandbox_pending``;
* ``ensure_sandbox(thread_id)`` — blocking 3-case lifecycle: no sandbox -> create (warm pool first) + claim;
  recorded + healthy -> reuse; recorded + unhealthy after ``restart_wait`` -> restart + claim;
* the claim config carries the thread's environment (THREAD_ID, USER_ID, KAFKA_PROFILE_ID, VM_API_KEY, MEMORY_DB_DSN,
  ...) like ``_build_claim_config`` in the reference.
Fixed vs the reference: the pending / ready maps are only mutated under an asyncio lock (SURVEY.md §5.2 lists the
unsynchronised fire-and-forget mutations as a latent race).

Provisioners (``sandbox/provisioner.py``): ``LocalProcessProvisioner`` spawns one ``sandbox/service.py`` process per
thread (own port + working directory); ``SharedURLProvisioner`` points every thread at one service URL.
"""
from __future__ import annotations

import asyncio
import logging
import os
from typing import Any

from kafka_llm_service_amd.sandbox.base import Sandbox, SandboxError

log = logging.getLogger("kafka.sandbox")


class SandboxManager:
    def __init__(self, db_client, provisioner, warm_factory=None, environment_id: str = "kafka-default",
                 health_timeout: float = 300.0, restart_wait: float = 60.0):
        self._db = db_client
        self._prov = provisioner
        self._warm = warm_factory
        self.environment_id = environment_id
        self.health_timeout = health_timeout
        self.restart_wait = restart_wait
        self._ready: dict[str, Sandbox] = {}
        self._pending: dict[str, asyncio.Task] = {}
        self._lock = asyncio.Lock()

    async def _build_claim_config(self, thread_id: str, sandbox_id: str) -> dict[str, Any]:
        cfg = await self._db.get_thread_config(thread_id) if hasattr(self._db, "get_thread_config") else None
        meta = (await self._db.get_thread_metadata(thread_id) or {}) if hasattr(self._db, "get_thread_metadata") \
            else {}
        user_id = (cfg or {}).get("user_id") or meta.get("user_id") or ""
        profile_id = (cfg or {}).get("kafka_profile_id") or meta.get("kafka_profile_id") or ""
        memory_dsn = (cfg or {}).get("memory_dsn") or os.getenv("MEMORY_DSN", "")
        vm_key = ""
        if hasattr(self._db, "get_or_create_vm_api_key"):
            vm_key = await self._db.get_or_create_vm_api_key(thread_id, user_id)
        return {"config": {"VM_API_KEY": vm_key or os.getenv("VM_API_KEY", "vm_dev_1234"), "USER_ID": str(user_id),
                           "KAFKA_PROFILE_ID": str(profile_id), "THREAD_ID": thread_id, "SANDBOX_ID": sandbox_id,
                           "DEV": os.getenv("DEV", "false"), "MEMORY_DB_DSN": memory_dsn}}

    async def _claim_if_needed(self, thread_id: str, sb: Sandbox, status: dict | None = None) -> None:
        status = status if status is not None else await sb.get_health_status()
        if status and not status.get("claimed"):
            await sb.claim(await self._build_claim_config(thread_id, sb.id))

    async def get_sandbox_if_ready(self, thread_id: str) -> Sandbox | None:
        sb = self._ready.get(thread_id)
        if sb is not None:
            status = await sb.get_health_status()
            if status and status.get("healthy"):
                await sb.check_health()
                await self._claim_if_needed(thread_id, sb, status)
                return sb
            async with self._lock:
                if self._ready.get(thread_id) is sb:
                    del self._ready[thread_id]  # stale
        if thread_id in self._pending:
            return None
        sid = await self._db.get_thread_sandbox_id(thread_id)
        if not sid:
            return None
        try:
            sb = await self._prov.connect(sid)
        except Exception:
            return None
        if sb is None or not await sb.check_health():
            return None
        await self._claim_if_needed(thread_id, sb)
        async with self._lock:
            self._ready[thread_id] = sb
        return sb

    def is_sandbox_pending(self, thread_id: str) -> bool:
        t = self._pending.get(thread_id)
        return t is not None and not t.done()

    def ensure_sandbox_background(self, thread_id: str) -> None:
        if self.is_sandbox_pending(thread_id) or thread_id in self._ready:
            return
        task = asyncio.get_running_loop().create_task(self._ensure_task(thread_id))
        self._pending[thread_id] = task

    async def _ensure_task(self, thread_id: str) -> None:
        try:
            await self.ensure_sandbox(thread_id)
        except Exception as e:
            log.warning("background sandbox for thread %s failed: %s", thread_id, e)
        finally:
            async with self._lock:
                self._pending.pop(thread_id, None)

    async def ensure_sandbox(self, thread_id: str) -> Sandbox:
        sb = await self.get_sandbox_if_ready(thread_id)
        if sb is not None:
            return sb
        sid = await self._db.get_thread_sandbox_id(thread_id)
        if sid:
            sb = await self._prov.connect(sid)
            if sb is not None:
                try:
                    await sb.wait_until_live(timeout=self.restart_wait)
                except SandboxError:
                    log.info("sandbox %s unhealthy; restarting", sid)
                    sb = await self._prov.restart(sid)
                    await sb.wait_until_live(timeout=self.health_timeout)
                await self._claim_if_needed(thread_id, sb)
                async with self._lock:
                    self._ready[thread_id] = sb
                return sb
        sb = await self._create_and_claim(thread_id)
        async with self._lock:
            self._ready[thread_id] = sb
        return sb

    async def _create_and_claim(self, thread_id: str) -> Sandbox:
        sb = None
        if self._warm is not None:
            sid = await self._warm.claim_sandbox(self.environment_id)
            if sid:
                sb = await self._prov.connect(sid)
        if sb is None:
            sb = await self._prov.create(thread_id)
        await self._db.update_thread_sandbox_id(thread_id, sb.id)
        await sb.wait_until_live(timeout=self.health_timeout)
        await self._claim_if_needed(thread_id, sb)
        return sb

    async def release_sandbox(self, thread_id: str) -> None:
        async with self._lock:
            sb = self._ready.pop(thread_id, None)
        if sb is not None:
            await self._prov.release(sb)

    async def shutdown(self) -> None:
        for t in list(self._pending.values()):
            t.cancel()
        for tid in list(self._ready):
            await self.release_sandbox(tid)
