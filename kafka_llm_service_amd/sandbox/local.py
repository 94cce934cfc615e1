"""HTTP client for a URL-addressed sandbox service (/root/reference/src/sandbox/local.py:18-386).

``wait_until_live`` polls ``/health`` every 2 s (default timeout 300 s); ``run_tool`` POSTs ``/run`` and parses
the SSE stream incrementally from raw bytes (line buffering would delay streamed shell output); ``claim`` POSTs the
per-thread environment. Transport failures surface as ``SandboxError``.
"""
from __future__ import annotations

import asyncio
import json
import time
from typing import Any, AsyncGenerator, Optional

import httpx

from kafka_llm_service_amd.utils import faults
from kafka_llm_service_amd.sandbox.base import Sandbox, SandboxError, SandboxInfo, SandboxState, ToolEvent


def parse_sse_event(line: str, tool_name: str) -> ToolEvent | None:
    """One ``data: ...`` line of the sandbox protocol -> ToolEvent (``[DONE]`` -> complete event)."""
    if not line.startswith("data:"):
        return None
    payload = line[5:].strip()
    if payload == "[DONE]":
        return ToolEvent(type="complete", data="", tool_name=tool_name, is_complete=True)
    try:
        d = json.loads(payload)
    except json.JSONDecodeError:
        return ToolEvent(type="output", data=payload, tool_name=tool_name)
    if not isinstance(d, dict):
        return ToolEvent(type="output", data=str(d), tool_name=tool_name)
    return ToolEvent(type=d.get("type", "output"), data=str(d.get("data", d.get("content", "")) or ""),
                     tool_name=tool_name, is_complete=bool(d.get("is_complete", False)),
                     exit_code=d.get("exit_code"), metadata=d.get("metadata") or {})


class LocalSandbox(Sandbox):
    DEFAULT_TIMEOUT = 300.0
    HEALTH_INTERVAL = 2.0

    def __init__(self, base_url: str, environment_id: str = "local", sandbox_id: str | None = None):
        super().__init__(sandbox_id or base_url, environment_id)
        self._base_url = base_url.rstrip("/")
        self._client: httpx.AsyncClient | None = None

    base_url = property(lambda self: self._base_url)
    health_url = property(lambda self: f"{self._base_url}/health")
    tool_run_url = property(lambda self: f"{self._base_url}/run")
    claim_url = property(lambda self: f"{self._base_url}/claim")

    async def _get_client(self) -> httpx.AsyncClient:
        if self._client is None or self._client.is_closed:
            self._client = httpx.AsyncClient(timeout=httpx.Timeout(self.DEFAULT_TIMEOUT))
        return self._client

    async def close(self) -> None:
        if self._client is not None:
            await self._client.aclose()
            self._client = None

    async def get_health_status(self) -> Optional[dict[str, Any]]:
        if faults.get().sandbox_down:
            return None
        try:
            r = await (await self._get_client()).get(self.health_url, timeout=5.0)
            if r.status_code == 200:
                return r.json()
        except (httpx.HTTPError, ValueError):
            return None
        return None

    async def check_health(self) -> bool:
        st = await self.get_health_status()
        ok = bool(st and st.get("healthy"))
        if ok:
            self._state = SandboxState.RUNNING
        return ok

    async def wait_until_live(self, timeout: Optional[float] = None) -> None:
        deadline = time.monotonic() + (timeout if timeout is not None else self.DEFAULT_TIMEOUT)
        self._state = SandboxState.STARTING if self._state != SandboxState.RUNNING else self._state
        while True:
            if await self.check_health():
                return
            if time.monotonic() >= deadline:
                self._state = SandboxState.ERROR
                raise SandboxError(f"sandbox not healthy after {timeout}s", self._id)
            await asyncio.sleep(min(self.HEALTH_INTERVAL, max(0.0, deadline - time.monotonic())))

    async def run_tool(self, tool_name: str, arguments: dict[str, Any]) -> AsyncGenerator[ToolEvent, None]:
        if faults.get().sandbox_down:
            raise SandboxError("Failed to connect to sandbox: injected fault (KAFKA_FI_SANDBOX_DOWN)", self._id)
        if self._state != SandboxState.RUNNING:
            raise SandboxError(f"Sandbox is not running (state: {self._state.value})", self._id)
        client = await self._get_client()
        try:
            async with client.stream("POST", self.tool_run_url, json={"tool_name": tool_name, "arguments": arguments},
                                     headers={"Accept": "text/event-stream"}) as resp:
                if resp.status_code != 200:
                    body = (await resp.aread()).decode(errors="replace")
                    raise SandboxError(f"Tool execution failed with status {resp.status_code}: {body}", self._id)
                buf = ""
                async for chunk in resp.aiter_bytes():
                    buf += chunk.decode("utf-8", errors="replace")
                    while "\n" in buf:
                        line, buf = buf.split("\n", 1)
                        ev = parse_sse_event(line.strip(), tool_name)
                        if ev is None:
                            continue
                        yield ev
                        if ev.is_complete:
                            return
        except httpx.ConnectError as e:
            raise SandboxError(f"Failed to connect to sandbox: {e}", self._id) from e
        except httpx.TimeoutException as e:
            raise SandboxError(f"Tool execution timed out: {e}", self._id) from e

    async def claim(self, data: dict[str, Any]) -> dict[str, Any]:
        try:
            r = await (await self._get_client()).post(self.claim_url, json=data, timeout=30.0)
        except httpx.HTTPError as e:
            raise SandboxError(f"claim failed: {e}", self._id) from e
        if r.status_code != 200:
            raise SandboxError(f"claim failed with status {r.status_code}: {r.text}", self._id)
        return r.json()

    async def reset(self) -> None:
        try:
            await (await self._get_client()).post(f"{self._base_url}/reset", timeout=30.0)
        except httpx.HTTPError:
            pass

    async def terminate(self) -> None:
        await self.close()
        self._state = SandboxState.TERMINATED

    async def get_info(self) -> SandboxInfo:
        return SandboxInfo(id=self._id, environment_id=self._environment_id, status=self._state.value,
                           url=self._base_url, metadata=self._metadata)

    @staticmethod
    async def connect(url: str, environment_id: str = "local") -> "LocalSandbox":
        sb = LocalSandbox(url, environment_id)
        await sb.check_health()
        return sb

    async def __aenter__(self) -> "LocalSandbox":
        return self

    async def __aexit__(self, *exc) -> None:
        await self.close()
