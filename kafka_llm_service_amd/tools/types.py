"""Tool types: local tools (sync / async / async-generator handlers), sandbox-forwarded tools, MCP server configs.

Behavioural parity with /root/reference/src/tools/types.py:23-463:
  * ``Tool.definition`` is the OpenAI function-calling schema; ``run`` folds a streaming handler, ``run_stream``
    yields a non-streaming handler's ``str(result)`` as one chunk (dict results are JSON-encoded here so the model sees
    valid JSON),
  * ``SandboxTool`` waits for its sandbox to be healthy (default 60 s) and forwards to ``sandbox.run_tool`` (SSE),
    yielding the ``data`` of every event,
  * ``ToolResultChunk`` is the unit the agent loop forwards as ``tool_result`` SSE frames.
"""
from __future__ import annotations

import asyncio
import inspect
import json
from typing import Any, AsyncGenerator, Callable, Optional, Union

from pydantic import BaseModel, Field

ToolHandler = Callable[..., Any]


class ToolProviderError(Exception):
    def __init__(self, message: str, tool_name: str | None = None, original_error: Exception | None = None):
        super().__init__(message)
        self.message = message
        self.tool_name = tool_name
        self.original_error = original_error

    def __str__(self) -> str:
        return f"[{self.tool_name}] {self.message}" if self.tool_name else self.message


class ToolResultChunk(BaseModel):
    delta: str = ""
    is_complete: bool = False
    tool_call_id: Optional[str] = None
    tool_name: Optional[str] = None


class ToolResult(BaseModel):
    success: bool
    result: Any = None
    error: Optional[str] = None


class MCPServerConfig(BaseModel):
    name: str
    command: Optional[str] = None
    args: list[str] = Field(default_factory=list)
    url: Optional[str] = None
    env: dict[str, str] = Field(default_factory=dict)


def _stringify(result: Any) -> str:
    if isinstance(result, str):
        return result
    if isinstance(result, (dict, list)):
        return json.dumps(result)
    return str(result)


class Tool:
    def __init__(self, name: str, description: str, parameters: dict[str, Any], handler: ToolHandler | None = None):
        self._name = name
        self._description = description
        self._parameters = parameters
        self._handler = handler

    name = property(lambda self: self._name)
    description = property(lambda self: self._description)
    parameters = property(lambda self: self._parameters)

    @property
    def definition(self) -> dict[str, Any]:
        return {"type": "function", "function": {"name": self._name, "description": self._description,
                                                 "parameters": self._parameters}}

    @property
    def has_handler(self) -> bool:
        return self._handler is not None

    @property
    def is_streaming(self) -> bool:
        return self._handler is not None and inspect.isasyncgenfunction(self._handler)

    def set_handler(self, handler: ToolHandler) -> None:
        self._handler = handler

    async def run(self, arguments: dict[str, Any]) -> Any:
        if self._handler is None:
            raise ToolProviderError(f"No handler registered for tool '{self._name}'", tool_name=self._name)
        if inspect.isasyncgenfunction(self._handler):
            return "".join([_stringify(c) async for c in self._handler(**arguments)])
        if asyncio.iscoroutinefunction(self._handler):
            return await self._handler(**arguments)
        res = self._handler(**arguments)
        if inspect.isawaitable(res):
            res = await res
        return res

    async def run_stream(self, arguments: dict[str, Any]) -> AsyncGenerator[str, None]:
        if self._handler is None:
            raise ToolProviderError(f"No handler registered for tool '{self._name}'", tool_name=self._name)
        if inspect.isasyncgenfunction(self._handler):
            async for chunk in self._handler(**arguments):
                yield _stringify(chunk)
            return
        yield _stringify(await self.run(arguments))

    def __repr__(self) -> str:
        return f"Tool(name={self._name!r})"


class SandboxTool:
    DEFAULT_HEALTH_TIMEOUT = 60.0

    def __init__(self, name: str, description: str, parameters: dict[str, Any], sandbox,
                 health_timeout: float | None = None):
        self._name = name
        self._description = description
        self._parameters = parameters
        self._sandbox = sandbox
        self._health_timeout = health_timeout or self.DEFAULT_HEALTH_TIMEOUT

    name = property(lambda self: self._name)
    description = property(lambda self: self._description)
    parameters = property(lambda self: self._parameters)
    sandbox = property(lambda self: self._sandbox)
    is_streaming = property(lambda self: True)

    @property
    def definition(self) -> dict[str, Any]:
        return {"type": "function", "function": {"name": self._name, "description": self._description,
                                                 "parameters": self._parameters}}

    async def _ensure_healthy(self) -> None:
        if not self._sandbox.is_running:
            await self._sandbox.wait_until_live(timeout=self._health_timeout)

    async def run(self, arguments: dict[str, Any]) -> str:
        return "".join([c async for c in self.run_stream(arguments)])

    async def run_stream(self, arguments: dict[str, Any]) -> AsyncGenerator[str, None]:
        await self._ensure_healthy()
        async for event in self._sandbox.run_tool(self._name, arguments):
            if event.data:
                yield event.data


AnyTool = Union[Tool, SandboxTool]
