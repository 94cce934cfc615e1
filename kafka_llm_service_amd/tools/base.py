"""ToolProvider: an ordered registry of local tools + MCP server configs (/root/reference/src/tools/base.py:73-245).

Tool order is insertion order and stays fixed for the life of the provider: the engine renders the tool schemas
into the prompt, so a stable order keeps the rendered system prefix byte-identical across requests and threads —
which is what makes it a prefix-cache hit.
"""
from __future__ import annotations

from typing import Any

from kafka_llm_service_amd.tools.types import MCPServerConfig, Tool, ToolProviderError


class ToolProvider:
    def __init__(self, tools: list[Tool] | None = None, mcp_servers: list[MCPServerConfig] | None = None):
        self._tools: dict[str, Any] = {}
        for t in tools or []:
            self.add_tool(t)
        self._mcp_servers: list[MCPServerConfig] = list(mcp_servers or [])

    @property
    def tools(self) -> list[Any]:
        return list(self._tools.values())

    @property
    def mcp_servers(self) -> list[MCPServerConfig]:
        return list(self._mcp_servers)

    def add_tool(self, tool) -> None:
        if tool.name in self._tools:
            raise ToolProviderError(f"Tool '{tool.name}' is already registered", tool_name=tool.name)
        self._tools[tool.name] = tool

    def remove_tool(self, name: str) -> bool:
        return self._tools.pop(name, None) is not None

    def get_tool(self, name: str):
        return self._tools.get(name)

    def has_tool(self, name: str) -> bool:
        return name in self._tools

    def add_mcp_server(self, config: MCPServerConfig) -> None:
        self._mcp_servers.append(config)

    async def get_tools(self) -> list[dict[str, Any]]:
        return [t.definition for t in self._tools.values()]

    async def run_tool(self, name: str, arguments: dict[str, Any]) -> Any:
        tool = self._tools.get(name)
        if tool is None:
            raise ToolProviderError(f"Unknown tool '{name}'", tool_name=name)
        return await tool.run(arguments)

    def __len__(self) -> int:
        return len(self._tools)

    def __contains__(self, name: str) -> bool:
        return name in self._tools
