"""Notebook tool forwarded to a sandbox (/root/reference/server_tools/notebook.py:15-107)."""
from __future__ import annotations

import os

from kafka_llm_service_amd.tools.types import MCPServerConfig, SandboxTool


class NotebookTools:
    def __init__(self, sandbox, health_timeout: int = 300):
        self.sandbox = sandbox
        self.health_timeout = health_timeout
        self.tools = [SandboxTool(
            "notebook_run_cell",
            "Execute Python code in a Jupyter-style notebook environment with persistent state between calls. Use it "
            "for data analysis, plotting, package installation and general Python execution. Output streams in "
            "real time as the code executes.",
            {"type": "object", "properties": {
                "code": {"type": "string", "description": "The Python code to execute in the notebook cell"},
                "description": {"type": "string", "description": "A brief description of what this code does"},
                "timeout": {"type": "integer", "description": "Maximum execution time in seconds (default: 3600)",
                            "default": 3600}}, "required": ["code", "description"]},
            sandbox, health_timeout)]


def get_notebook_mcp_server() -> MCPServerConfig:
    """Deprecated path kept for parity: the notebook as a stdio MCP server (NOTEBOOK_MCP_SERVER_PATH)."""
    path = os.environ.get("NOTEBOOK_MCP_SERVER_PATH", "notebook_mcp_server.py")
    return MCPServerConfig(name="notebook", command="python", args=[path],
                           env={"EXEC_DIR": os.environ.get("EXEC_DIR", os.getcwd())})
