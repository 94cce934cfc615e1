"""Sandbox service + client + manager + lazy sandbox, shell / notebook tools, MCP stdio client (CPU, local
processes only)."""
import asyncio
import os
import socket
import subprocess
import sys

import pytest

from kafka_llm_service_amd.db.local import MemoryDBClient
from kafka_llm_service_amd.sandbox.lazy import LazySandbox
from kafka_llm_service_amd.sandbox.local import LocalSandbox, parse_sse_event
from kafka_llm_service_amd.sandbox.manager import SandboxManager
from kafka_llm_service_amd.sandbox.provisioner import LocalProcessProvisioner
from kafka_llm_service_amd.server_tools import NotebookTools, ShellTools
from kafka_llm_service_amd.tools.agent import AgentToolProvider
from kafka_llm_service_amd.tools.mcp import MCPConnection
from kafka_llm_service_amd.tools.types import MCPServerConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def sandbox_url(tmp_path_factory):
    port = _port()
    wd = tmp_path_factory.mktemp("sbx")
    p = subprocess.Popen([sys.executable, "-m", "kafka_llm_service_amd.sandbox.service", "--port", str(port),
                          "--workdir", str(wd)], cwd=ROOT)
    url = f"http://127.0.0.1:{port}"
    yield url
    p.terminate()
    p.wait(10)


async def _collect(agen):
    return [x async for x in agen]


def test_sse_parser():
    assert parse_sse_event('data: {"type":"output","data":"x"}', "t").data == "x"
    assert parse_sse_event("data: [DONE]", "t").is_complete
    assert parse_sse_event("event: ping", "t") is None
    assert parse_sse_event("data: not json", "t").data == "not json"


def test_shell_and_notebook_through_tools(sandbox_url):
    async def main():
        sb = LocalSandbox(sandbox_url)
        await sb.wait_until_live(timeout=60)
        st = await sb.get_health_status()
        assert st["healthy"] and not st["claimed"]
        await sb.claim({"config": {"THREAD_ID": "t1"}})
        assert (await sb.get_health_status())["claimed"]
        tp = AgentToolProvider(sandbox_tools=ShellTools(sb).tools + NotebookTools(sb).tools)
        await tp.connect()
        out = await _collect(tp.run_tool_stream("shell_exec", {"shell_id": "nope", "command": "ls"}, "c0"))
        assert "create_shell" in out[0].delta
        await _collect(tp.run_tool_stream("create_shell", {"shell_id": "main"}, "c1"))
        await _collect(tp.run_tool_stream("shell_exec", {"shell_id": "main", "command": "cd /tmp && export Z=42"},
                                          "c2"))
        out = await _collect(tp.run_tool_stream("shell_exec", {"shell_id": "main", "command": "pwd; echo $Z $THREAD_ID"},
                                                "c3"))
        text = "".join(c.delta for c in out)
        assert "/tmp" in text and "42 t1" in text and out[-1].is_complete and out[-1].delta == ""
        await _collect(tp.run_tool_stream("notebook_run_cell", {"code": "x = 6 * 7", "description": "d"}, "c4"))
        out = await _collect(tp.run_tool_stream("notebook_run_cell", {"code": "print(x)\nx + 1", "description": "d"},
                                                "c5"))
        text = "".join(c.delta for c in out)
        assert "42" in text and "43" in text
        out = await _collect(tp.run_tool_stream("notebook_run_cell", {"code": "1/0", "description": "d"}, "c6"))
        assert "ZeroDivisionError" in "".join(c.delta for c in out)
        await sb.close()
    asyncio.run(main())


def test_manager_lazy_and_process_provisioner(tmp_path):
    async def main():
        db = MemoryDBClient()
        await db.initialize()
        t = await db.create_thread(user_id="u9")
        prov = LocalProcessProvisioner(root=str(tmp_path))
        mgr = SandboxManager(db, prov, health_timeout=60)
        try:
            assert await mgr.get_sandbox_if_ready(t["id"]) is None
            lazy = LazySandbox(t["id"], mgr, timeout=60)
            mgr.ensure_sandbox_background(t["id"])
            assert mgr.is_sandbox_pending(t["id"])
            tools = ShellTools(lazy).tools
            evs = await _collect(tools[0].run_stream({"shell_id": "s"}))
            assert "created" in "".join(evs)
            evs = await _collect(tools[1].run_stream({"shell_id": "s", "command": "echo $THREAD_ID $USER_ID"}))
            assert f"{t['id']} u9" in "".join(evs)
            sid = await db.get_thread_sandbox_id(t["id"])
            assert sid and sid.startswith("http://")
            assert (await mgr.get_sandbox_if_ready(t["id"])) is not None
        finally:
            await mgr.shutdown()
            prov.shutdown()
    asyncio.run(main())


def test_mcp_stdio_client_and_routing():
    async def main():
        cfg = MCPServerConfig(name="echo", command=sys.executable,
                              args=[os.path.join(ROOT, "tests", "fixtures", "mcp_echo_server.py")])
        conn = MCPConnection(cfg, timeout=30)
        await conn.connect()
        assert [t["function"]["name"] for t in conn.tools] == ["echo", "add"]
        assert await conn.call_tool("add", {"a": 2, "b": 3}) == "5"
        await conn.disconnect()
        tp = AgentToolProvider(mcp_servers=[cfg, MCPServerConfig(name="dead", url="http://127.0.0.1:9/mcp")])
        await tp.connect()  # the unreachable server is skipped
        names = [t["function"]["name"] for t in await tp.get_tools()]
        assert names == ["echo", "add"] and tp.tool_source("echo") == "echo"
        out = await _collect(tp.run_tool_stream("echo", {"text": "hey"}, "c1"))
        assert out[0].delta == "hey" and out[-1].is_complete
        await tp.disconnect()
    asyncio.run(main())


def test_daytona_sandbox_interface_offline():
    """Daytona sandboxes are LocalSandboxes addressed by id; lifecycle calls need the SDK and say so."""
    import asyncio

    from kafka_llm_service_amd.sandbox.base import SandboxError
    from kafka_llm_service_amd.sandbox.daytona import DaytonaSandbox

    sb = DaytonaSandbox("abc123", "env")
    assert sb.base_url == "https://8081-abc123.proxy.daytona.works" and sb.id == "abc123"
    assert sb.health_url.endswith("/health") and sb.tool_run_url.endswith("/run")
    try:
        asyncio.run(DaytonaSandbox.create("snap"))
        raise AssertionError("expected SandboxError")
    except SandboxError as e:
        assert "daytona_sdk" in str(e)


def test_mcp_http_falls_back_to_legacy_sse():
    """A URL server that refuses streamable HTTP is reached over the legacy HTTP+SSE transport
    (/root/reference/src/tools/agent.py:113-162)."""
    import socket
    import subprocess
    import time

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    proc = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "fixtures", "mcp_sse_server.py"),
                             str(port)])
    try:
        import httpx

        for _ in range(100):
            try:
                httpx.post(f"http://127.0.0.1:{port}/sse", timeout=1)
                break
            except httpx.HTTPError:
                time.sleep(0.1)

        async def main():
            conn = MCPConnection(MCPServerConfig(name="legacy", url=f"http://127.0.0.1:{port}/sse"), timeout=20)
            await conn.connect()
            assert type(conn._t).__name__ == "_SseTransport"
            assert [t["function"]["name"] for t in conn.tools] == ["echo", "add"]
            assert await conn.call_tool("add", {"a": 4, "b": 5}) == "9"
            assert await conn.call_tool("echo", {"text": "over sse"}) == "over sse"
            await conn.disconnect()
        asyncio.run(main())
    finally:
        proc.terminate()
        proc.wait(timeout=10)
