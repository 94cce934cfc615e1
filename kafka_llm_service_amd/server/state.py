"""Server configuration and lifespan state (the wiring the reference does in ``lifespan``, server.py:89-150).

``ServerConfig.from_env`` keeps the reference's variable names where they still apply (PORT, DEFAULT_MODEL,
LOCAL_SANDBOX_URL, LOCAL_DB_PATH) and adds the engine's:
  KAFKA_LLM_BACKEND   engine | stub            (stub = instant echo provider, BASELINE config 1)
  KAFKA_MODEL         llama3-8b | llama3-70b | mixtral-8x7b | tiny-llama | <HF dir>
  KAFKA_WEIGHTS       safetensors dir (default: seeded random init)
  KAFKA_DP / KAFKA_TP data-parallel replicas / tensor-parallel size (one worker process per GPU)
  KAFKA_SANDBOX       shared | process | none   (shared = one sandbox service at LOCAL_SANDBOX_URL)
  KAFKA_MCP           1 to connect DEFAULT_MCP_SERVERS (off by default: the hosts are offline)
"""
from __future__ import annotations

import logging
import json
import os
from dataclasses import dataclass, field
from typing import Any, AsyncGenerator

from kafka_llm_service_amd.kafka.v1 import KafkaV1Provider
from kafka_llm_service_amd.llm.types import Message

log = logging.getLogger("kafka.server")


@dataclass
class ServerConfig:
    backend: str = "engine"
    model: str = "llama3-8b"
    weights: str | None = None
    served_model_name: str | None = None
    dp: int = 1
    tp: int = 1
    db: str = "local"                    # "local" (SQLite, LOCAL_DB_PATH) | "supabase" (SUPABASE_URL / SUPABASE_KEY)
    db_path: str = "data/threads.db"
    sandbox: str = "shared"
    sandbox_url: str = "http://localhost:8081"
    mcp: bool = False
    max_model_len: int = 131072
    default_max_tokens: int = 1024
    # default tool_choice of engine-backed generations ("auto" | "required" | "none" | a JSON function object);
    # "required" makes random-init models drive the agent/tool loop with well-formed calls (BASELINE config 4). A
    # LIST is a per-iteration script: agent iteration i of a turn (i = assistant tool-call messages since the last
    # user message) uses entry min(i, len - 1), e.g. create_shell, then shell_exec, then get_weather
    tool_choice: Any = "auto"
    # JSON-schema overrides of tool parameters by tool name (KAFKA_TOOL_OVERRIDES, a JSON object): e.g. enum values
    # that pin a random-init model's constrained arguments to a working call ({"shell_id": {"enum": ["main"]}})
    tool_overrides: dict[str, Any] = field(default_factory=dict)
    # subset of the Kafka v1 prompt sections (None = all 13: the reference's 70,496-character prompt, or ~47k with
    # KAFKA_PROMPT=compact); small engines / CPU tests use a few
    prompt_sections: list[str] | None = None
    agent_max_iterations: int = 50  # LLM <-> tool rounds per agent run (the reference's Agent default, base.py:78)
    warm_prefix: bool = True  # prefill + pin the shared system prefix on every replica before serving
    ignore_eos: bool = False  # benchmarks: generate exactly max_tokens (random-init weights emit EOS at random)
    # run a single engine in its own worker process (like a DP replica) instead of a thread of the API process: the
    # step loop's kernel launches then never compete with the HTTP/SSE event loop for the GIL
    engine_process: bool = False
    # Mixtral: the ``dp`` replicas form one data-parallel-attention EP group (engine/dp_attention.py)
    dp_attention: bool = False
    engine_kwargs: dict[str, Any] = field(default_factory=dict)

    @staticmethod
    def from_env() -> "ServerConfig":
        e = os.environ
        return ServerConfig(backend=e.get("KAFKA_LLM_BACKEND", "engine"), model=e.get("KAFKA_MODEL", "llama3-8b"),
                            weights=e.get("KAFKA_WEIGHTS") or None,
                            served_model_name=e.get("DEFAULT_MODEL") or None, dp=int(e.get("KAFKA_DP", "1")),
                            tp=int(e.get("KAFKA_TP", "1")), db_path=e.get("LOCAL_DB_PATH", "data/threads.db"),
                            db=e.get("KAFKA_DB", "local"),
                            sandbox=e.get("KAFKA_SANDBOX", "shared"),
                            sandbox_url=e.get("LOCAL_SANDBOX_URL", "http://localhost:8081"),
                            mcp=e.get("KAFKA_MCP", "0") == "1",
                            max_model_len=int(e.get("KAFKA_MAX_MODEL_LEN", "131072")),
                            default_max_tokens=int(e.get("KAFKA_DEFAULT_MAX_TOKENS", "1024")),
                            tool_choice=_tool_choice(e.get("KAFKA_TOOL_CHOICE", "auto")),
                            tool_overrides=json.loads(e.get("KAFKA_TOOL_OVERRIDES", "{}")),
                            ignore_eos=e.get("KAFKA_IGNORE_EOS", "0") == "1",
                            warm_prefix=e.get("KAFKA_WARM_PREFIX", "1") == "1",
                            engine_process=_engine_process(e.get("KAFKA_ENGINE_PROCESS", "auto")),
                            dp_attention=e.get("KAFKA_DP_ATTENTION", "0") == "1",
                            prompt_sections=[x for x in e.get("KAFKA_PROMPT_SECTIONS", "").split(",") if x] or None,
                            agent_max_iterations=int(e.get("KAFKA_AGENT_MAX_ITERATIONS", "50")),
                            engine_kwargs=_engine_kwargs(e))


def _engine_kwargs(e) -> dict[str, Any]:
    """Engine options from the environment: KAFKA_KV_DTYPE (bf16 | fp8 KV cache), KAFKA_GRAPHS=1 (hipGraph decode
    steps), KAFKA_MAX_NUM_SEQS, KAFKA_MAX_BATCHED_TOKENS."""
    kw: dict[str, Any] = {}
    if e.get("KAFKA_KV_DTYPE"):
        kw["kv_dtype"] = e["KAFKA_KV_DTYPE"]
    if e.get("KAFKA_GRAPHS") in ("0", "1"):  # unset: the engine's default (on for TP > 1)
        kw["use_graphs"] = e["KAFKA_GRAPHS"] == "1"
    if e.get("KAFKA_MAX_NUM_SEQS"):
        kw["max_num_seqs"] = int(e["KAFKA_MAX_NUM_SEQS"])
    if e.get("KAFKA_MAX_BATCHED_TOKENS"):  # prefill tokens per step (smaller: earlier first tokens in a burst)
        kw["max_num_batched_tokens"] = kw["max_prefill_chunk"] = int(e["KAFKA_MAX_BATCHED_TOKENS"])
    return kw


def _engine_process(v: str) -> bool:
    """auto: a GPU server runs its engine in a worker process (measured on MI355X, 64 threads: p50 TTFT 125 ms vs
    242 ms with the step loop sharing the API process's GIL — profiles/serve_bench_engine_gpu_r01.log)."""
    if v == "auto":
        import torch

        return torch.cuda.device_count() > 0
    return v == "1"


def apply_tool_overrides(tools: list, overrides: dict[str, Any]) -> list:
    """Tools with ``overrides[name]`` ({property: JSON schema}) merged into their parameters' properties — copies,
    so module-level tool singletons stay untouched."""
    if not overrides:
        return list(tools)
    import copy

    out = []
    for t in tools:
        ov = overrides.get(t.name)
        if ov:
            t = copy.copy(t)
            params = copy.deepcopy(t.parameters)
            params.setdefault("properties", {}).update(copy.deepcopy(ov))
            t._parameters = params
        out.append(t)
    return out


def _tool_choice(v: str) -> Any:
    v = v.strip()
    return json.loads(v) if v.startswith(("{", "[")) else v


class ServerState:
    def __init__(self, config: ServerConfig, llm_provider=None, db=None):
        self.config = config
        self.llm = llm_provider
        self.db = db
        self.engine_client = None
        self.kafka: KafkaV1Provider | None = None
        self.sandbox_manager = None
        self.global_sandbox = None
        self.provisioner = None
        self.ready = False

    # ------------------------------------------------------------------------------------------------------------
    async def start(self) -> None:
        from kafka_llm_service_amd.db.local import LocalDBClient
        from kafka_llm_service_amd.server_tools import (DEFAULT_MCP_SERVERS, NotebookTools, PlannerTools, ShellTools,
                                                        count_tool, get_weather_tool)

        cfg = self.config
        if self.db is None:
            if cfg.db == "supabase":
                from kafka_llm_service_amd.db.supabase import SupabaseDBClient

                self.db = SupabaseDBClient()
            else:
                self.db = LocalDBClient(cfg.db_path)
        await self.db.initialize()
        if self.llm is None:
            self.llm = await self._make_llm()
        sandbox_tools = []
        if cfg.sandbox != "none":
            from kafka_llm_service_amd.sandbox.local import LocalSandbox
            from kafka_llm_service_amd.sandbox.manager import SandboxManager
            from kafka_llm_service_amd.sandbox.provisioner import (HTTPWarmSandboxFactory, LocalProcessProvisioner,
                                                                   SharedURLProvisioner)

            self.global_sandbox = LocalSandbox(cfg.sandbox_url)
            sandbox_tools = ShellTools(self.global_sandbox).tools + NotebookTools(self.global_sandbox).tools
            self.provisioner = LocalProcessProvisioner() if cfg.sandbox == "process" else \
                SharedURLProvisioner(cfg.sandbox_url)
            warm = HTTPWarmSandboxFactory() if os.environ.get("WARM_SANDBOX_SERVICE_URL") else None
            self.sandbox_manager = SandboxManager(self.db, self.provisioner, warm)
        tools = apply_tool_overrides([get_weather_tool, count_tool] + PlannerTools(None).tools, cfg.tool_overrides)
        sandbox_tools = apply_tool_overrides(sandbox_tools, cfg.tool_overrides)
        self.kafka = KafkaV1Provider(self.llm, tools=tools, sandbox_tools=sandbox_tools,
                                     mcp_servers=DEFAULT_MCP_SERVERS if cfg.mcp else [],
                                     prompt_sections=cfg.prompt_sections, max_iterations=cfg.agent_max_iterations)
        await self.kafka.initialize()
        if cfg.backend == "engine" and cfg.warm_prefix and hasattr(self.llm, "warm") and self.kafka.system_prompt:
            n = await self.llm.warm(self.kafka.system_prompt, await self.kafka.get_tools())
            log.info("shared system prefix prefilled and pinned: %d tokens", n)
        self.ready = True
        log.info("server ready (backend=%s model=%s)", cfg.backend, cfg.model)

    async def _make_llm(self):
        cfg = self.config
        if cfg.backend == "stub":
            from kafka_llm_service_amd.llm.stub import StubEchoProvider

            return StubEchoProvider()
        if cfg.backend == "remote":  # chain to another OpenAI-compatible server (KAFKA_REMOTE_URL / _MODEL)
            from kafka_llm_service_amd.llm.remote import RemoteOpenAIProvider

            return RemoteOpenAIProvider(os.environ["KAFKA_REMOTE_URL"], os.environ.get("KAFKA_REMOTE_MODEL", cfg.model),
                                        default_max_tokens=cfg.default_max_tokens)
        from kafka_llm_service_amd.engine.client import make_engine_client
        from kafka_llm_service_amd.llm.engine_provider import EngineLLMProvider

        self.engine_client = await make_engine_client(cfg)
        return EngineLLMProvider(self.engine_client, default_max_tokens=cfg.default_max_tokens,
                                 model_name=self.model_ids()[0], tool_choice=cfg.tool_choice,
                                 ignore_eos=cfg.ignore_eos)

    async def stop(self) -> None:
        self.ready = False
        if self.kafka is not None:
            await self.kafka.cleanup()
        if self.sandbox_manager is not None:
            await self.sandbox_manager.shutdown()
        if self.provisioner is not None and hasattr(self.provisioner, "shutdown"):
            self.provisioner.shutdown()
        if self.global_sandbox is not None:
            await self.global_sandbox.close()
        if self.engine_client is not None:
            await self.engine_client.close()
        if self.db is not None:
            await self.db.close()

    # ------------------------------------------------------------------------------------------------------------
    def model_ids(self) -> list[str]:
        name = self.config.served_model_name or self.config.model
        return [name]

    def engine_health(self) -> dict[str, Any]:
        if self.engine_client is None:
            return {"backend": self.config.backend}
        return self.engine_client.health()

    async def run_agent(self, messages: list[Message], model: str, temperature: float | None,
                        max_tokens: int | None, thread_id: str | None, **kw) -> AsyncGenerator[dict, None]:
        """The global agent (reference: ``kafka.run`` for /chat/completions and /agent/run); with a thread id the
        history is loaded and the turn persisted (quirk Q3 fix: the reference never persisted tool turns here)."""
        temp = 0.7 if temperature is None else temperature
        if thread_id is None:
            async for ev in self.kafka.run(messages, model=model, temperature=temp, max_tokens=max_tokens, **kw):
                yield ev
            return
        async for ev in self.kafka.run_with_thread(messages, model=model, temperature=temp, max_tokens=max_tokens,
                                                   thread_id=thread_id, db_client=self.db, routing_key=thread_id,
                                                   **kw):
            yield ev

    async def run_thread_agent(self, thread_id: str, messages: list[Message], model: str, temperature: float,
                               max_tokens: int | None) -> AsyncGenerator[dict, None]:
        """Per-thread agent: thread profile prompt + playbooks, per-thread planner state, the thread's own sandbox
        resolved lazily (reference: generate_agent_stream_with_thread, server.py:204-263)."""
        from kafka_llm_service_amd.server_tools import NotebookTools, PlannerTools, ShellTools, count_tool, \
            get_weather_tool

        sandbox_tools = []
        if self.sandbox_manager is not None:
            from kafka_llm_service_amd.sandbox.lazy import LazySandbox

            sb = await self.sandbox_manager.get_sandbox_if_ready(thread_id)
            if sb is None:
                self.sandbox_manager.ensure_sandbox_background(thread_id)
                sb = LazySandbox(thread_id, self.sandbox_manager, timeout=120.0)
            sandbox_tools = ShellTools(sb).tools + NotebookTools(sb).tools
        ov = self.config.tool_overrides
        agent = KafkaV1Provider(self.llm, thread_id=thread_id, db_client=self.db,
                                tools=apply_tool_overrides([get_weather_tool, count_tool] + PlannerTools(thread_id).tools,
                                                           ov),
                                sandbox_tools=apply_tool_overrides(sandbox_tools, ov),
                                prompt_sections=self.config.prompt_sections,
                                max_iterations=self.config.agent_max_iterations)
        await agent.initialize()
        try:
            async for ev in agent.run_with_thread(messages, model=model, temperature=temperature,
                                                  max_tokens=max_tokens, routing_key=thread_id):
                yield ev
        finally:
            await agent.cleanup()
