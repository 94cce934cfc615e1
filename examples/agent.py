#!/usr/bin/env python3
"""Example Kafka v1 agent on the on-node engine (the reference's examples/agent.py demo, re-done for this stack).

Builds an engine client (in-process, one GPU — or CPU with the tiny test model), wraps it in the engine-backed
LLMProvider and runs a KafkaV1Provider agent with the weather and counter tools, printing the live event stream.
Random-init weights never choose a tool on their own, so ``--tool-choice required`` forces a (schema-valid) call.

  python examples/agent.py --model tiny-llama --device cpu --tool-choice required --prompt-sections intro,core_tools
  python examples/agent.py --model llama3-8b                       # GPU 0, random-init Llama-3-8B
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from kafka_llm_service_amd.engine.client import InProcessClient  # noqa: E402
from kafka_llm_service_amd.engine.engine import EngineConfig  # noqa: E402
from kafka_llm_service_amd.kafka.v1 import KafkaV1Provider  # noqa: E402
from kafka_llm_service_amd.llm.engine_provider import EngineLLMProvider  # noqa: E402
from kafka_llm_service_amd.llm.types import Message  # noqa: E402
from kafka_llm_service_amd.server_tools import count_tool, get_weather_tool  # noqa: E402


async def main(args) -> int:
    os.environ.setdefault("KAFKA_WEATHER_MODE", "offline")
    kw = {"device": args.device} if args.device else {}
    if args.device == "cpu":
        kw["num_kv_blocks"] = 4096
    client = await asyncio.to_thread(InProcessClient, EngineConfig(model=args.model, max_model_len=32768, **kw))
    tc = json.loads(args.tool_choice) if args.tool_choice.startswith("{") else args.tool_choice
    llm = EngineLLMProvider(client, default_max_tokens=args.max_tokens, model_name=args.model, tool_choice=tc,
                            ignore_eos=True)
    sections = [x for x in args.prompt_sections.split(",") if x] or None
    agent = KafkaV1Provider(llm, tools=[get_weather_tool, count_tool], max_iterations=args.max_iterations,
                            prompt_sections=sections)
    await agent.initialize()
    print(f"user: {args.prompt}\nagent:")
    n_tool = 0
    try:
        async for ev in agent.run([Message(role="user", content=args.prompt)], model=args.model,
                                  temperature=args.temperature):
            if ev.get("object") == "chat.completion.chunk":
                d = ev["choices"][0]["delta"]
                if d.get("content"):
                    print(d["content"], end="", flush=True)
                for tc in d.get("tool_calls") or []:
                    f = tc.get("function") or {}
                    if f.get("name"):
                        print(f"\n[tool call] {f['name']}", end="")
                    if f.get("arguments"):
                        print(f" {f['arguments']}", end="")
            elif ev.get("type") == "tool_result":
                n_tool += 1
                if ev["delta"]:
                    print(f"\n[tool result] {ev['delta']}", end="")
            elif ev.get("type") == "agent_done":
                print(f"\n[done] {json.dumps({k: v for k, v in ev.items() if k != 'type'})}")
    finally:
        await agent.cleanup()
        await client.close()
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--device", default=None)
    ap.add_argument("--prompt", default="What's the weather like in Tokyo?")
    ap.add_argument("--tool-choice", default="auto")
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--max-tokens", type=int, default=48)
    ap.add_argument("--max-iterations", type=int, default=3)
    ap.add_argument("--prompt-sections", default="", help="comma-separated subset of the Kafka prompt sections")
    sys.exit(asyncio.run(main(ap.parse_args())))
