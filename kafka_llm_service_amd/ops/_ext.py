"""Loader for the in-tree HIP kernel extension ``_kafka_ops.so``.

On a GPU process the extension is mandatory: if it is missing or fails to load, every GPU op raises instead of
silently falling back to PyTorch. CPU tensors use ``ops.reference`` (tests / CPU-only runs).
"""
from __future__ import annotations

import importlib
import os
from pathlib import Path

_EXT = None
_ERR: Exception | None = None


def load(build_if_missing: bool = True):
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    import torch  # noqa: F401  (torch's HIP runtime must be loaded before our .so)

    so = Path(__file__).with_name("_kafka_ops.so")
    if not so.exists() and build_if_missing and os.environ.get("KAFKA_NO_BUILD") != "1":
        from kafka_llm_service_amd.ops import build as _b

        _b.build()
    try:
        _EXT = importlib.import_module("kafka_llm_service_amd.ops._kafka_ops")
    except Exception as e:  # pragma: no cover - exercised on broken builds only
        _ERR = e
        raise RuntimeError(f"kafka HIP extension failed to load from {so}: {e}") from e
    return _EXT


def ext():
    return _EXT if _EXT is not None else load()
