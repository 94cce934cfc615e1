"""AgentToolProvider: one tool namespace over local tools, MCP-server tools and sandbox tools.

Routing parity with /root/reference/src/tools/agent.py:416-833:
  * ``connect()`` connects every MCP server (a failing server is skipped with a warning), maps each discovered tool
    to its server, and marks local ("local") and sandbox ("sandbox") tools,
  * ``get_tools()`` lists regular tools, then MCP tools, then sandbox tools — a fixed order (prefix-cache friendly),
  * ``run_tool_stream()`` yields ``ToolResultChunk`` deltas and ALWAYS ends with an empty ``is_complete=True``
    chunk; unknown tools / missing handlers / exceptions become a single ``"Error: ..."`` complete chunk.
"""
from __future__ import annotations

import logging
from typing import Any, AsyncGenerator

from kafka_llm_service_amd.tools.base import ToolProvider
from kafka_llm_service_amd.tools.mcp import MCPConnection
from kafka_llm_service_amd.tools.types import MCPServerConfig, SandboxTool, Tool, ToolResultChunk

log = logging.getLogger("kafka.tools")

BROADCAST_PIPE = "/tmp/kafka_broadcaster_pipe"


def _as_tool(t) -> Tool:
    if isinstance(t, dict):
        fn = t.get("function", t)
        return Tool(fn["name"], fn.get("description", ""), fn.get("parameters", {}))
    return t


class AgentToolProvider(ToolProvider):
    def __init__(self, tools: list | None = None, mcp_servers: list | None = None,
                 sandbox_tools: list[SandboxTool] | None = None, broadcast_pipe: str | None = BROADCAST_PIPE):
        servers = [s if isinstance(s, MCPServerConfig) else MCPServerConfig(**s) for s in (mcp_servers or [])]
        self._tool_source_map: dict[str, str] = {}
        super().__init__(tools=[_as_tool(t) for t in (tools or [])], mcp_servers=servers)
        self._mcp_connections: dict[str, MCPConnection] = {}
        self._sandbox_tools: dict[str, SandboxTool] = {st.name: st for st in (sandbox_tools or [])}
        self._connected = False
        self.broadcast_pipe = broadcast_pipe

    def register_handler(self, name: str, handler) -> None:
        tool = self.get_tool(name)
        if tool is not None:
            tool.set_handler(handler)
        self._tool_source_map[name] = "local"

    def add_tool(self, tool) -> None:
        super().add_tool(tool)
        self._tool_source_map.setdefault(tool.name, "local")

    async def connect(self) -> None:
        for cfg in self._mcp_servers:
            try:
                conn = MCPConnection(cfg)
                await conn.connect()
                self._mcp_connections[cfg.name] = conn
                for t in conn.tools:
                    self._tool_source_map[t["function"]["name"]] = cfg.name
            except Exception as e:  # the reference logs and continues (src/tools/agent.py:494-496)
                log.warning("failed to connect to MCP server %s: %s", cfg.name, e)
        for name in self._tools:
            self._tool_source_map.setdefault(name, "local")
        for name in self._sandbox_tools:
            self._tool_source_map[name] = "sandbox"
        self._connected = True

    async def disconnect(self) -> None:
        for conn in self._mcp_connections.values():
            await conn.disconnect()
        self._mcp_connections.clear()

    @property
    def is_connected(self) -> bool:
        return self._connected

    async def get_tools(self) -> list[dict[str, Any]]:
        out = [t.definition for t in self._tools.values()]
        for conn in self._mcp_connections.values():
            out.extend(conn.tools)
        out.extend(st.definition for st in self._sandbox_tools.values())
        return out

    def add_sandbox_tool(self, tool: SandboxTool) -> None:
        self._sandbox_tools[tool.name] = tool
        self._tool_source_map[tool.name] = "sandbox"

    def get_sandbox_tool(self, name: str) -> SandboxTool | None:
        return self._sandbox_tools.get(name)

    def has_tool(self, name: str) -> bool:
        return name in self._tool_source_map or name in self._tools or name in self._sandbox_tools

    def tool_source(self, name: str) -> str | None:
        return self._tool_source_map.get(name)

    async def run_tool(self, name: str, arguments: dict[str, Any]) -> Any:
        src = self._tool_source_map.get(name, "local" if name in self._tools else None)
        if src == "sandbox":
            return await self._sandbox_tools[name].run(arguments)
        if src == "local":
            return await super().run_tool(name, arguments)
        if src in self._mcp_connections:
            return await self._mcp_connections[src].call_tool(name, arguments)
        raise KeyError(f"Tool not found: {name}")

    async def run_tool_stream(self, name: str, arguments: dict[str, Any],
                              tool_call_id: str) -> AsyncGenerator[ToolResultChunk, None]:
        def chunk(delta: str, done: bool) -> ToolResultChunk:
            return ToolResultChunk(tool_call_id=tool_call_id, tool_name=name, delta=delta, is_complete=done)

        src = self._tool_source_map.get(name)
        if src is None and name in self._tools:
            src = "local"
        if src is None:
            yield chunk(f"Error: Tool not found: {name}", True)
            return
        try:
            if src == "sandbox":
                st = self._sandbox_tools.get(name)
                if st is None:
                    yield chunk(f"Error: Sandbox tool not found: {name}", True)
                    return
                stream = st.run_stream(arguments)
            elif src == "local":
                tool = self.get_tool(name)
                if tool is None or not tool.has_handler:
                    yield chunk(f"Error: Tool not found or no handler: {name}", True)
                    return
                stream = tool.run_stream(arguments)
            else:
                conn = self._mcp_connections.get(src)
                if conn is None:
                    yield chunk(f"Error: MCP server not connected: {src}", True)
                    return
                stream = conn.call_tool_stream(name, arguments, self.broadcast_pipe)
            async for delta in stream:
                yield chunk(delta, False)
            yield chunk("", True)
        except Exception as e:
            yield chunk(f"Error: {e}", True)
