"""Sequential-thinking planner tools: ``sequentialthinking``, ``saveThoughtCheckpoint``, ``loadThoughtCheckpoint``.

State machine parity with /root/reference/server_tools/planner.py:14-307 (thought history, branches, goal summary,
plan + updated plan, checkpoints; JSON results). Fixed (quirk Q9): the reference kept ONE process-global state shared
by every thread; here ``PlannerTools(thread_id)`` gets the thread's own state from a registry.
"""
from __future__ import annotations

import json
import threading
from typing import Any

from kafka_llm_service_amd.tools.types import Tool


class SequentialThinkingServer:
    def __init__(self):
        self.thought_history: list[dict[str, Any]] = []
        self.branches: dict[str, list[dict[str, Any]]] = {}
        self.goal_summary = ""
        self.current_plan: list[dict[str, Any]] = []
        self.checkpoints: dict[str, dict[str, Any]] = {}

    def process_thought(self, **kw) -> str:
        n = int(kw.get("thoughtNumber", 1))
        total = max(int(kw.get("totalThoughts", 1)), n)
        if n == 1 and kw.get("goalSummary"):
            self.goal_summary = kw["goalSummary"]
        if n == 1 and kw.get("plan"):
            self.current_plan = list(kw["plan"])
        if kw.get("updatedPlan"):
            self.current_plan = list(kw["updatedPlan"])
        t = {"thought": kw.get("thought", ""), "thoughtNumber": n, "totalThoughts": total,
             "nextThoughtNeeded": bool(kw.get("nextThoughtNeeded", True)), "isRevision": kw.get("isRevision", False),
             "revisesThought": kw.get("revisesThought"), "branchFromThought": kw.get("branchFromThought"),
             "branchId": kw.get("branchId"), "needsMoreThoughts": kw.get("needsMoreThoughts", False),
             "goalSummary": kw.get("goalSummary"), "completedStep": kw.get("completedStep")}
        self.thought_history.append(t)
        if t["branchFromThought"] and t["branchId"]:
            self.branches.setdefault(t["branchId"], []).append(t)
        return json.dumps({
            "thoughtNumber": n, "totalThoughts": total, "nextThoughtNeeded": t["nextThoughtNeeded"],
            "branches": list(self.branches), "thoughtHistoryLength": len(self.thought_history),
            "goalSummary": self.goal_summary, "currentPlan": self.current_plan,
            "completedStep": t["completedStep"], "previousThoughts": self.thought_history[-3:],
            "thoughtHistory": [{"thought": x["thought"], "thoughtNumber": x["thoughtNumber"],
                                "isRevision": x.get("isRevision"), "branchId": x.get("branchId"),
                                "completedStep": x.get("completedStep")} for x in self.thought_history]}, indent=2)

    def save_checkpoint(self, checkpointId: str | None = None) -> str:
        cid = checkpointId or f"checkpoint_{len(self.checkpoints)}"
        self.checkpoints[cid] = {"thoughtHistory": list(self.thought_history), "branches": dict(self.branches),
                                 "goalSummary": self.goal_summary, "currentPlan": list(self.current_plan)}
        return json.dumps({"result": f"Checkpoint {cid} saved successfully", "checkpointId": cid}, indent=2)

    def load_checkpoint(self, checkpointId: str) -> str:
        if checkpointId not in self.checkpoints:
            return json.dumps({"error": f"Checkpoint {checkpointId} not found"}, indent=2)
        c = self.checkpoints[checkpointId]
        self.thought_history = list(c["thoughtHistory"])
        self.branches = dict(c["branches"])
        self.goal_summary = c["goalSummary"]
        self.current_plan = list(c["currentPlan"])
        return json.dumps({"result": f"Checkpoint {checkpointId} loaded successfully",
                           "thoughtHistory": self.thought_history, "goalSummary": self.goal_summary,
                           "currentPlan": self.current_plan}, indent=2)


_REGISTRY: dict[str, SequentialThinkingServer] = {}
_REG_LOCK = threading.Lock()


def server_for(thread_id: str | None) -> SequentialThinkingServer:
    key = thread_id or "__global__"
    with _REG_LOCK:
        if key not in _REGISTRY:
            _REGISTRY[key] = SequentialThinkingServer()
        return _REGISTRY[key]


_PLAN_ITEM = {"type": "object", "properties": {"text": {"type": "string"}, "completed": {
    "type": "string", "enum": ["true", "false", "in progress"]}}, "required": ["text", "completed"]}


class PlannerTools:
    def __init__(self, thread_id: str | None = None):
        self.thread_id = thread_id
        self.server = server_for(thread_id)
        s = self.server
        self.tools = [
            Tool("sequentialthinking",
                 "Plan and reason step by step. Each call records one thought; keep a goal summary and a plan with "
                 "per-step completion state, revise or branch earlier thoughts when new information arrives, and "
                 "set nextThoughtNeeded=false when the plan is complete.",
                 {"type": "object", "properties": {
                     "thought": {"type": "string", "description": "Your current thinking step"},
                     "goalSummary": {"type": "string", "description": "Summary of the overall goal (first thought)"},
                     "plan": {"type": "array", "items": _PLAN_ITEM, "description": "Initial plan (first thought)"},
                     "updatedPlan": {"type": "array", "items": _PLAN_ITEM, "description": "Revised plan"},
                     "completedStep": {"type": "string", "description": "Plan step completed by this thought"},
                     "nextThoughtNeeded": {"type": "boolean", "description": "Whether another thought is needed"},
                     "thoughtNumber": {"type": "integer", "description": "Current thought number", "minimum": 1},
                     "totalThoughts": {"type": "integer", "description": "Estimated total thoughts", "minimum": 1},
                     "isRevision": {"type": "boolean", "description": "Whether this revises previous thinking"},
                     "revisesThought": {"type": "integer", "description": "Which thought is being reconsidered"},
                     "branchFromThought": {"type": "integer", "description": "Branching point thought number"},
                     "branchId": {"type": "string", "description": "Branch identifier"},
                     "needsMoreThoughts": {"type": "boolean", "description": "If more thoughts are needed"}},
                  "required": ["thought", "nextThoughtNeeded", "thoughtNumber", "totalThoughts"]},
                 handler=lambda **kw: s.process_thought(**kw)),
            Tool("saveThoughtCheckpoint", "Save the current thinking state to a checkpoint for later retrieval",
                 {"type": "object", "properties": {"checkpointId": {
                     "type": "string", "description": "Optional checkpoint identifier"}}, "required": []},
                 handler=lambda checkpointId=None: s.save_checkpoint(checkpointId)),
            Tool("loadThoughtCheckpoint", "Load a previously saved thinking state from a checkpoint",
                 {"type": "object", "properties": {"checkpointId": {
                     "type": "string", "description": "Checkpoint identifier to load"}}, "required": ["checkpointId"]},
                 handler=lambda checkpointId: s.load_checkpoint(checkpointId)),
        ]
