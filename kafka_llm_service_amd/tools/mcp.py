"""Minimal Model Context Protocol client (JSON-RPC 2.0) — stdio, streamable HTTP, and the legacy HTTP+SSE
transport as the fallback for URL servers that do not speak streamable HTTP.

The reference drives MCP servers through the ``mcp`` SDK (/root/reference/src/tools/agent.py:63-413: stdio or
streamable-HTTP with SSE fallback, ``tools/list`` discovery, ``tools/call``, and a streaming side channel that tails
NDJSON ``{"delta": {"content": ...}}`` lines from a named pipe while the call runs). The SDK is not installable here,
so this module speaks the protocol directly: ``initialize`` -> ``notifications/initialized`` -> ``tools/list`` /
``tools/call``. Connection failures are reported to the caller, which (like the reference) skips that server.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import os
from typing import Any, AsyncGenerator

from kafka_llm_service_amd.tools.types import MCPServerConfig

PROTOCOL_VERSION = "2025-03-26"
CLIENT_INFO = {"name": "kafka-llm-service-amd", "version": "1.0"}


class MCPError(Exception):
    pass


def _mcp_tool_to_openai(t: dict) -> dict:
    return {"type": "function", "function": {"name": t["name"], "description": t.get("description", ""),
                                             "parameters": t.get("inputSchema") or {"type": "object",
                                                                                   "properties": {}}}}


def _result_text(result: dict) -> str:
    parts = []
    for block in result.get("content", []) or []:
        if block.get("type") == "text":
            parts.append(block.get("text", ""))
        else:
            parts.append(json.dumps(block))
    text = "\n".join(parts)
    if result.get("isError"):
        return f"Error: {text}"
    return text


class _StdioTransport:
    def __init__(self, cfg: MCPServerConfig):
        self.cfg = cfg
        self.proc: asyncio.subprocess.Process | None = None
        self.pending: dict[int, asyncio.Future] = {}
        self.reader_task: asyncio.Task | None = None

    async def start(self) -> None:
        env = dict(os.environ)
        env.update(self.cfg.env or {})
        self.proc = await asyncio.create_subprocess_exec(self.cfg.command, *(self.cfg.args or []),
                                                         stdin=asyncio.subprocess.PIPE,
                                                         stdout=asyncio.subprocess.PIPE,
                                                         stderr=asyncio.subprocess.DEVNULL, env=env)
        self.reader_task = asyncio.create_task(self._read_loop())

    async def _read_loop(self) -> None:
        assert self.proc and self.proc.stdout
        while True:
            line = await self.proc.stdout.readline()
            if not line:
                break
            try:
                msg = json.loads(line)
            except json.JSONDecodeError:
                continue
            fut = self.pending.pop(msg.get("id"), None) if "id" in msg else None
            if fut is not None and not fut.done():
                fut.set_result(msg)
        for fut in self.pending.values():
            if not fut.done():
                fut.set_exception(MCPError("MCP server closed the connection"))

    async def request(self, msg: dict, timeout: float) -> dict | None:
        assert self.proc and self.proc.stdin
        fut = None
        if "id" in msg:
            fut = asyncio.get_running_loop().create_future()
            self.pending[msg["id"]] = fut
        self.proc.stdin.write((json.dumps(msg) + "\n").encode())
        await self.proc.stdin.drain()
        if fut is None:
            return None
        return await asyncio.wait_for(fut, timeout)

    async def close(self) -> None:
        if self.reader_task:
            self.reader_task.cancel()
        if self.proc and self.proc.returncode is None:
            self.proc.terminate()
            try:
                await asyncio.wait_for(self.proc.wait(), 5)
            except asyncio.TimeoutError:
                self.proc.kill()


class _HttpTransport:
    """Streamable HTTP: POST JSON-RPC, the response is either JSON or an SSE stream carrying the reply."""

    def __init__(self, cfg: MCPServerConfig):
        self.cfg = cfg
        self.session_id: str | None = None
        self.client = None

    async def start(self) -> None:
        import httpx

        self.client = httpx.AsyncClient(timeout=60.0)

    async def request(self, msg: dict, timeout: float) -> dict | None:
        headers = {"Accept": "application/json, text/event-stream", "Content-Type": "application/json"}
        if self.session_id:
            headers["Mcp-Session-Id"] = self.session_id
        r = await self.client.post(self.cfg.url, content=json.dumps(msg), headers=headers, timeout=timeout)
        if r.status_code >= 400:
            raise MCPError(f"MCP HTTP {r.status_code}: {r.text[:200]}")
        self.session_id = r.headers.get("mcp-session-id", self.session_id)
        if "id" not in msg:
            return None
        ctype = r.headers.get("content-type", "")
        if "text/event-stream" in ctype:
            for line in r.text.splitlines():
                if line.startswith("data:"):
                    try:
                        data = json.loads(line[5:].strip())
                    except json.JSONDecodeError:
                        continue
                    if data.get("id") == msg["id"]:
                        return data
            raise MCPError("no JSON-RPC reply in SSE response")
        return r.json()

    async def close(self) -> None:
        if self.client:
            await self.client.aclose()


def _message_url(base: str, endpoint: str) -> str:
    from urllib.parse import urljoin

    return urljoin(base, endpoint)


class _SseTransport:
    """Legacy HTTP+SSE (MCP 2024-11-05): GET the server URL as an event stream; its first ``endpoint`` event names
    the URL to POST JSON-RPC messages to; replies arrive as ``message`` events on the stream. A reader task routes
    them to the waiting requests by id."""

    def __init__(self, cfg: MCPServerConfig):
        self.cfg = cfg
        self.client = None
        self.post_url: str | None = None
        self.pending: dict[int, asyncio.Future] = {}
        self.reader_task: asyncio.Task | None = None
        self._endpoint: asyncio.Future | None = None

    async def start(self, timeout: float = 30.0) -> None:
        import httpx

        self.client = httpx.AsyncClient(timeout=httpx.Timeout(timeout, read=None))
        self._endpoint = asyncio.get_running_loop().create_future()
        self.reader_task = asyncio.create_task(self._read_loop())
        self.post_url = await asyncio.wait_for(self._endpoint, timeout)

    async def _read_loop(self) -> None:
        event, data = "message", []
        try:
            async with self.client.stream("GET", self.cfg.url, headers={"Accept": "text/event-stream"}) as r:
                if r.status_code >= 400:
                    raise MCPError(f"MCP SSE HTTP {r.status_code}")
                async for line in r.aiter_lines():
                    if line.startswith("event:"):
                        event = line[6:].strip()
                    elif line.startswith("data:"):
                        data.append(line[5:].strip())
                    elif not line:  # end of one event
                        self._dispatch(event, "\n".join(data))
                        event, data = "message", []
        except Exception as e:  # noqa: BLE001 - surfaced to every waiter
            err = e if isinstance(e, MCPError) else MCPError(f"MCP SSE stream failed: {e!r}")
            if self._endpoint is not None and not self._endpoint.done():
                self._endpoint.set_exception(err)
            for fut in self.pending.values():
                if not fut.done():
                    fut.set_exception(err)
            return
        for fut in self.pending.values():
            if not fut.done():
                fut.set_exception(MCPError("MCP SSE stream closed"))

    def _dispatch(self, event: str, data: str) -> None:
        if event == "endpoint":
            if not self._endpoint.done():
                self._endpoint.set_result(_message_url(self.cfg.url, data))
            return
        try:
            msg = json.loads(data)
        except json.JSONDecodeError:
            return
        fut = self.pending.pop(msg.get("id"), None) if isinstance(msg, dict) else None
        if fut is not None and not fut.done():
            fut.set_result(msg)

    async def request(self, msg: dict, timeout: float) -> dict | None:
        fut = None
        if "id" in msg:
            fut = asyncio.get_running_loop().create_future()
            self.pending[msg["id"]] = fut
        r = await self.client.post(self.post_url, content=json.dumps(msg),
                                   headers={"Content-Type": "application/json"}, timeout=timeout)
        if r.status_code >= 400:
            self.pending.pop(msg.get("id"), None)
            raise MCPError(f"MCP SSE POST {r.status_code}: {r.text[:200]}")
        if fut is None:
            return None
        return await asyncio.wait_for(fut, timeout)

    async def close(self) -> None:
        if self.reader_task:
            self.reader_task.cancel()
            try:
                await self.reader_task
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        if self.client:
            await self.client.aclose()


class MCPConnection:
    def __init__(self, config: MCPServerConfig, timeout: float = 60.0):
        self.config = config
        self.timeout = timeout
        self.tools: list[dict] = []
        self._ids = itertools.count(1)
        self._t = None
        self.connected = False

    async def connect(self) -> None:
        """stdio for a command; for a URL streamable HTTP first and, if the server does not answer it, the legacy
        HTTP+SSE transport (the fallback order of /root/reference/src/tools/agent.py:113-162)."""
        if self.config.command:
            self._t = _StdioTransport(self.config)
            await self._t.start()
            await self._handshake()
        elif self.config.url:
            self._t = _HttpTransport(self.config)
            await self._t.start()
            try:
                await self._handshake()
            except Exception as first:  # noqa: BLE001
                await self._t.close()
                self._t = _SseTransport(self.config)
                try:
                    await self._t.start(min(self.timeout, 30.0))
                    await self._handshake()
                except Exception as e:  # noqa: BLE001
                    await self._t.close()
                    raise MCPError(f"MCP {self.config.name!r}: streamable HTTP failed ({first}); SSE failed ({e})")
        else:
            raise MCPError(f"MCP server {self.config.name!r} has neither command nor url")
        self.connected = True

    async def _handshake(self) -> None:
        await self._rpc("initialize", {"protocolVersion": PROTOCOL_VERSION, "capabilities": {},
                                       "clientInfo": CLIENT_INFO})
        await self._t.request({"jsonrpc": "2.0", "method": "notifications/initialized"}, self.timeout)
        res = await self._rpc("tools/list", {})
        self.tools = [_mcp_tool_to_openai(t) for t in res.get("tools", [])]

    async def _rpc(self, method: str, params: dict) -> dict:
        msg = {"jsonrpc": "2.0", "id": next(self._ids), "method": method, "params": params}
        reply = await self._t.request(msg, self.timeout)
        if reply is None:
            raise MCPError("no reply")
        if "error" in reply:
            raise MCPError(f"{method}: {reply['error'].get('message', reply['error'])}")
        return reply.get("result", {})

    async def call_tool(self, name: str, arguments: dict[str, Any]) -> str:
        return _result_text(await self._rpc("tools/call", {"name": name, "arguments": arguments}))

    async def call_tool_stream(self, name: str, arguments: dict[str, Any],
                               broadcast_pipe: str | None = None) -> AsyncGenerator[str, None]:
        """Yield streamed deltas from the NDJSON side channel while the call runs; fall back to the final result."""
        if not broadcast_pipe or not os.path.exists(broadcast_pipe):
            yield await self.call_tool(name, arguments)
            return
        q: asyncio.Queue = asyncio.Queue()
        done = asyncio.Event()

        async def tail():
            fd = os.open(broadcast_pipe, os.O_RDONLY | os.O_NONBLOCK)
            buf = b""
            try:
                while not done.is_set():
                    try:
                        data = os.read(fd, 65536)
                    except BlockingIOError:
                        data = b""
                    if data:
                        buf += data
                        while b"\n" in buf:
                            line, buf = buf.split(b"\n", 1)
                            try:
                                delta = json.loads(line).get("delta", {}).get("content")
                            except (json.JSONDecodeError, AttributeError):
                                delta = None
                            if delta:
                                await q.put(delta)
                    else:
                        await asyncio.sleep(0.01)
            finally:
                os.close(fd)

        tail_task = asyncio.create_task(tail())
        call_task = asyncio.create_task(self.call_tool(name, arguments))
        got = False
        while not call_task.done() or not q.empty():
            try:
                item = await asyncio.wait_for(q.get(), 0.05)
                got = True
                yield item
            except asyncio.TimeoutError:
                continue
        done.set()
        await tail_task
        result = await call_task
        if not got:
            yield result

    async def disconnect(self) -> None:
        if self._t:
            await self._t.close()
        self.connected = False
