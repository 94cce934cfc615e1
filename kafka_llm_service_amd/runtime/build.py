"""Build the native host runtime ``_kafka_runtime.so`` (C++17 + pybind11, no torch dependency) in-tree.

Run ``python -m kafka_llm_service_amd.runtime.build``. ``KAFKA_SANITIZE=1`` builds it with
``-fsanitize=address,undefined`` (host code only) into ``_kafka_runtime_asan.so``.
"""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pybind11

from kafka_llm_service_amd.utils.native_build import Unit, build_shared, python_include

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"


def build(verbose: bool = False, sanitize: bool | None = None) -> Path:
    sanitize = os.environ.get("KAFKA_SANITIZE") == "1" if sanitize is None else sanitize
    flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"-I{pybind11.get_include()}",
             f"-I{python_include()}", "-Wall", "-Wno-unused-function"]
    link = []
    name = "_kafka_runtime"
    if sanitize:
        flags = [f for f in flags if f != "-O2"] + ["-O1", "-g", "-fsanitize=address,undefined",
                                                    "-fno-omit-frame-pointer"]
        link = ["-fsanitize=address,undefined"]
        name = "_kafka_runtime_asan"
    units = [Unit(p, "g++", flags) for p in sorted(CSRC.glob("*.cpp"))]
    bdir = HERE / (".build_asan" if sanitize else ".build")
    return build_shared(units, HERE / f"{name}.so", link, "g++", bdir, verbose=verbose)


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
