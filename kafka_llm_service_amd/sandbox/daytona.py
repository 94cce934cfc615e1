"""Daytona cloud sandboxes (/root/reference/src/sandbox/daytona.py:38-575) — interface kept, cloud optional.

A Daytona sandbox speaks exactly the local sandbox protocol (``/health``, ``/claim``, ``/run`` SSE) at
``https://8081-{sandbox_id}.proxy.daytona.works``, so ``DaytonaSandbox`` is a ``LocalSandbox`` addressed by id.
Lifecycle calls (create from a snapshot + fire-and-forget ``./start.sh``, restart of a stopped sandbox) need the
``daytona_sdk`` package and network access; neither exists on this machine, so they raise ``SandboxError`` with a
clear message when the SDK is missing ("Drop (cloud-only); interface kept"). The local
provisioners in ``sandbox/provisioner.py`` are what the server uses here.
"""
from __future__ import annotations

import asyncio
import os
from typing import Optional

from kafka_llm_service_amd.sandbox.base import SandboxError, SandboxState
from kafka_llm_service_amd.sandbox.local import LocalSandbox

PROXY_TEMPLATE = os.environ.get("DAYTONA_PROXY_TEMPLATE", "https://8081-{id}.proxy.daytona.works")
STARTUP_CMD = "nohup ./start.sh > /log.txt 2>&1 &"


def _sdk():
    try:
        import daytona_sdk  # noqa: F401
    except ImportError as e:
        raise SandboxError("Daytona sandboxes need the daytona_sdk package (not installed here); use the local "
                           "sandbox service / provisioners instead", "daytona") from e
    key = os.environ.get("DAYTONA_API_KEY")
    if not key:
        raise SandboxError("DAYTONA_API_KEY is not set", "daytona")
    from daytona_sdk import Daytona, DaytonaConfig

    return Daytona(DaytonaConfig(api_key=key))


class DaytonaSandbox(LocalSandbox):
    def __init__(self, sandbox_id: str, environment_id: str = "unknown"):
        super().__init__(PROXY_TEMPLATE.format(id=sandbox_id), environment_id, sandbox_id=sandbox_id)

    @staticmethod
    async def create(environment_id: str, auto_stop_interval: int = 0,
                     env_vars: Optional[dict[str, str]] = None) -> "DaytonaSandbox":
        """Create from a snapshot, start its services in the background; call ``wait_until_live`` next."""
        client = _sdk()
        from daytona_sdk import CreateSandboxFromSnapshotParams

        try:
            sb = await asyncio.to_thread(client.create, CreateSandboxFromSnapshotParams(
                public=True, auto_stop_interval=auto_stop_interval, snapshot=environment_id))
        except Exception as e:
            raise SandboxError(f"Failed to create Daytona sandbox: {e}", "daytona") from e
        asyncio.create_task(asyncio.to_thread(sb.process.exec, STARTUP_CMD, "/", env_vars or {}))
        out = DaytonaSandbox(sb.id, environment_id)
        out._state = SandboxState.STARTING
        return out

    @staticmethod
    async def restart_sandbox(sandbox_id: str, environment_id: str = "unknown") -> "DaytonaSandbox":
        client = _sdk()
        try:
            sb = await asyncio.to_thread(client.get, sandbox_id)
            if getattr(sb, "state", None) != "started":
                await asyncio.to_thread(sb.start)
            await asyncio.to_thread(sb.process.exec, STARTUP_CMD, "/")
        except Exception as e:
            raise SandboxError(f"Failed to restart Daytona sandbox {sandbox_id}: {e}", sandbox_id) from e
        out = DaytonaSandbox(sandbox_id, environment_id)
        out._state = SandboxState.STARTING
        return out

    @staticmethod
    async def connect(sandbox_id: str, environment_id: str = "unknown") -> "DaytonaSandbox":
        """Attach to an existing sandbox by id (no SDK needed: the proxy URL is derived from the id)."""
        sb = DaytonaSandbox(sandbox_id, environment_id)
        await sb.check_health()
        return sb
