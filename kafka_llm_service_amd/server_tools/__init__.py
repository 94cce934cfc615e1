"""Server tool catalog (/root/reference/server_tools/__init__.py:8-24)."""
from kafka_llm_service_amd.server_tools.counter import count_tool
from kafka_llm_service_amd.server_tools.mcp_servers import DEFAULT_MCP_SERVERS
from kafka_llm_service_amd.server_tools.notebook import NotebookTools
from kafka_llm_service_amd.server_tools.planner import PlannerTools
from kafka_llm_service_amd.server_tools.shell import ShellTools
from kafka_llm_service_amd.server_tools.weather import get_weather_tool

__all__ = ["count_tool", "get_weather_tool", "ShellTools", "NotebookTools", "PlannerTools", "DEFAULT_MCP_SERVERS"]
