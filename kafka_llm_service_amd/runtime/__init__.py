"""Native host runtime (C++): KV block manager + prefix cache. Built in-tree by ``runtime/build.py``."""
from __future__ import annotations

import importlib
import os
from pathlib import Path

_MOD = None


def native():
    """Import ``_kafka_runtime`` (building it first if it is missing and building is allowed)."""
    global _MOD
    if _MOD is not None:
        return _MOD
    so = Path(__file__).with_name("_kafka_runtime.so")
    if not so.exists() and os.environ.get("KAFKA_NO_BUILD") != "1":
        from . import build as _b

        _b.build()
    _MOD = importlib.import_module("kafka_llm_service_amd.runtime._kafka_runtime")
    return _MOD


def KVManager(num_blocks: int, page: int = 16, prefix_cache: bool = True, run: int = 1):
    return native().KVManager(num_blocks, page, prefix_cache, run)
