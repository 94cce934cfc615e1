"""Shell tools forwarded to a sandbox (/root/reference/server_tools/shell.py:14-75)."""
from __future__ import annotations

from kafka_llm_service_amd.tools.types import SandboxTool


class ShellTools:
    def __init__(self, sandbox, health_timeout: int = 30):
        self.sandbox = sandbox
        self.health_timeout = health_timeout
        self.tools = [
            SandboxTool("create_shell", "Create a new shell session in the sandbox. You must create a shell before "
                        "running commands.",
                        {"type": "object", "properties": {"shell_id": {
                            "type": "string", "description": "A unique identifier for the shell session (e.g., "
                                                             "'main', 'worker1')"}}, "required": ["shell_id"]},
                        sandbox, health_timeout),
            SandboxTool("shell_exec", "Execute a shell command in an existing shell session. Returns the command "
                        "output.",
                        {"type": "object", "properties": {
                            "shell_id": {"type": "string", "description": "The shell session ID to run the command in"},
                            "command": {"type": "string", "description": "The shell command to execute"}},
                         "required": ["shell_id", "command"]}, sandbox, health_timeout),
        ]
