"""``count_slowly``: streaming demo tool (async generator handler; /root/reference/server_tools/counter.py:13-44)."""
from __future__ import annotations

import asyncio

from kafka_llm_service_amd.tools.types import Tool


async def count_slowly(count: int = 10, delay: float = 1.0):
    for i in range(1, int(count) + 1):
        await asyncio.sleep(float(delay))
        yield f"{i}... "
    yield "Done!"


count_tool = Tool(
    name="count_slowly",
    description="Count from 1 to a number slowly, with a delay between each number. Useful for demonstrating "
                "streaming tool results.",
    parameters={"type": "object", "properties": {
        "count": {"type": "integer", "description": "The number to count to. Defaults to 10.", "default": 10},
        "delay": {"type": "number", "description": "Seconds between each number. Defaults to 1.0.", "default": 1.0}},
        "required": []},
    handler=count_slowly)
