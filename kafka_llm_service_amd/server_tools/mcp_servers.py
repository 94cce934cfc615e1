"""Default MCP servers (/root/reference/server_tools/mcp_servers.py:8-13). Remote servers are unreachable offline;
AgentToolProvider.connect skips a server it cannot reach, exactly like the reference."""
from kafka_llm_service_amd.tools.types import MCPServerConfig

DEFAULT_MCP_SERVERS = [MCPServerConfig(name="fetch", url="https://remote.mcpservers.org/fetch/mcp")]
