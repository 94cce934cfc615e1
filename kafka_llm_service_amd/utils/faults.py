"""Fault injection ("fault-injection env flags (KAFKA_FI_*: drop sandbox, slow step, OOM)").

The reference has no fault injection at all (its failure handling is sandbox health polling and per-server MCP
tolerance). Every hook here is off unless its environment variable is set, and costs one attribute
check when off:

  KAFKA_FI_SLOW_STEP_MS=<ms>      every engine step sleeps this long first (stall / watchdog tests)
  KAFKA_FI_STEP_ERROR_EVERY=<n>   every n-th engine step raises InjectedFault (in-flight requests must fail cleanly,
                                  the engine must keep serving new ones)
  KAFKA_FI_WORKER_EXIT_AFTER=<n>  a DP/TP worker process hard-exits after n steps (replica crash -> 503-style errors
                                  for its streams, re-route, respawn)
  KAFKA_FI_KV_BLOCKS=<n>          cap the KV page pool (memory pressure -> preemption by recompute)
  KAFKA_FI_SANDBOX_DOWN=1         sandbox health checks and tool calls fail (error tool_result frames)
  KAFKA_FI_CAR_SKIP_CALL=<n>      this rank skips its n-th custom xGMI all-reduce call (a peer that stops arriving:
                                  its peers' waits time out and the TP leader's engine must raise, not emit tokens)
"""
from __future__ import annotations

import os
import time


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, env: dict | None = None):
        e = os.environ if env is None else env
        self.slow_step_s = float(e.get("KAFKA_FI_SLOW_STEP_MS", "0") or 0) / 1e3
        self.step_error_every = int(e.get("KAFKA_FI_STEP_ERROR_EVERY", "0") or 0)
        self.worker_exit_after = int(e.get("KAFKA_FI_WORKER_EXIT_AFTER", "0") or 0)
        kv = e.get("KAFKA_FI_KV_BLOCKS")
        self.kv_blocks = int(kv) if kv else None
        self.sandbox_down = e.get("KAFKA_FI_SANDBOX_DOWN", "0") == "1"
        self.car_skip_call = int(e.get("KAFKA_FI_CAR_SKIP_CALL", "0") or 0)
        self.active = bool(self.slow_step_s or self.step_error_every or self.worker_exit_after or self.kv_blocks
                           or self.sandbox_down or self.car_skip_call)
        self._steps = 0

    def on_step(self) -> None:
        """Called at the top of every engine step."""
        self._steps += 1
        if self.slow_step_s:
            time.sleep(self.slow_step_s)
        if self.step_error_every and self._steps % self.step_error_every == 0:
            raise InjectedFault(f"injected engine step failure (step {self._steps})")

    def worker_should_exit(self, steps: int) -> bool:
        return bool(self.worker_exit_after) and steps >= self.worker_exit_after


_FI: FaultInjector | None = None


def get() -> FaultInjector:
    global _FI
    if _FI is None:
        _FI = FaultInjector()
    return _FI


def reset(env: dict | None = None) -> FaultInjector:
    """Re-read the flags (tests)."""
    global _FI
    _FI = FaultInjector(env)
    return _FI
