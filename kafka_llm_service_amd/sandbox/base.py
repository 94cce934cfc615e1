"""Sandbox interface (/root/reference/src/sandbox/base.py:15-267, types.py:10-70).

A sandbox is an isolated execution environment reachable over the sandbox HTTP protocol:
``GET /health -> {"healthy", "claimed"}``, ``POST /claim {"config": {...env}}``, ``POST /run {"tool_name",
"arguments"}`` -> SSE ``data: {"type", "data", "is_complete", "exit_code", "metadata"}`` ... ``data: [DONE]``.
``sandbox/service.py`` is this repo's implementation of that service (the reference relied on Daytona VMs).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from enum import Enum
from typing import Any, AsyncGenerator, Optional

from pydantic import BaseModel, Field


class SandboxState(Enum):
    CREATING = "creating"
    STARTING = "starting"
    RUNNING = "running"
    STOPPED = "stopped"
    ERROR = "error"
    TERMINATED = "terminated"
    UNKNOWN = "unknown"


class SandboxError(Exception):
    def __init__(self, message: str, sandbox_id: Optional[str] = None):
        super().__init__(message)
        self.message = message
        self.sandbox_id = sandbox_id

    def __str__(self) -> str:
        return f"[sandbox {self.sandbox_id}] {self.message}" if self.sandbox_id else self.message


class SandboxConfig(BaseModel):
    environment_id: str
    timeout: int = 300
    metadata: dict[str, Any] = Field(default_factory=dict)


class SandboxInfo(BaseModel):
    id: str
    environment_id: str
    status: str
    created_at: Optional[str] = None
    url: Optional[str] = None
    metadata: dict[str, Any] = Field(default_factory=dict)


class ToolEvent(BaseModel):
    type: str
    data: str = ""
    tool_name: str
    is_complete: bool = False
    exit_code: Optional[int] = None
    metadata: dict[str, Any] = Field(default_factory=dict)


class Sandbox(ABC):
    def __init__(self, sandbox_id: str, environment_id: str):
        self._id = sandbox_id
        self._environment_id = environment_id
        self._state = SandboxState.UNKNOWN
        self._metadata: dict[str, Any] = {}

    @property
    def id(self) -> str:
        return self._id

    @property
    def environment_id(self) -> str:
        return self._environment_id

    @property
    def state(self) -> SandboxState:
        return self._state

    @property
    def is_running(self) -> bool:
        return self._state == SandboxState.RUNNING

    @property
    def metadata(self) -> dict[str, Any]:
        return self._metadata

    @abstractmethod
    async def check_health(self) -> bool: ...

    @abstractmethod
    async def get_health_status(self) -> Optional[dict[str, Any]]: ...

    @abstractmethod
    async def wait_until_live(self, timeout: Optional[float] = None) -> None: ...

    @abstractmethod
    def run_tool(self, tool_name: str, arguments: dict[str, Any]) -> AsyncGenerator[ToolEvent, None]: ...

    @abstractmethod
    async def claim(self, data: dict[str, Any]) -> dict[str, Any]: ...

    async def stop(self) -> None:
        self._state = SandboxState.STOPPED

    async def reset(self) -> None:
        pass

    async def terminate(self) -> None:
        self._state = SandboxState.TERMINATED

    async def get_info(self) -> SandboxInfo:
        return SandboxInfo(id=self._id, environment_id=self._environment_id, status=self._state.value,
                           metadata=self._metadata)

    def __repr__(self) -> str:
        return f"{self.__class__.__name__}(id={self._id!r}, state={self._state.value})"
