"""Build the CDNA4 kernel extension ``_kafka_ops.so`` in-tree.

Kernel translation units (``csrc/*.hip``) are compiled by hipcc for gfx950 only and include nothing from torch;
``csrc/bindings.cpp`` is the only torch-aware unit (host code, compiled with g++ against torch's headers so the
C++ ABI matches libtorch). Run ``python -m kafka_llm_service_amd.ops.build``.
"""
from __future__ import annotations

import sys
from pathlib import Path

from kafka_llm_service_amd.utils.native_build import (ARCH, ROCM, Unit, build_shared, hipcc, python_include,
                                                      torch_paths)

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
OUT = HERE / "_kafka_ops.so"

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-fgpu-flush-denormals-to-zero", "-Wno-unused-result"]


def build(verbose: bool = False) -> Path:
    troot, tincs, abi = torch_paths()
    units = [Unit(p, hipcc(), HIP_FLAGS) for p in sorted(CSRC.glob("*.hip"))]
    bind_flags = ["-O2", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-D__HIP_PLATFORM_AMD__=1",
                  "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_kafka_ops", "-DTORCH_API_INCLUDE_EXTENSION_H",
                  f"-I{ROCM / 'include'}", f"-I{python_include()}", *[f"-I{p}" for p in tincs],
                  "-Wno-deprecated-declarations"]
    units.append(Unit(CSRC / "bindings.cpp", "g++", bind_flags))
    tlib = troot / "lib"
    link = [f"--offload-arch={ARCH}", f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
            "-ltorch_python", f"-Wl,-rpath,{tlib}", "-Wl,--no-undefined" if False else "-Wl,-O1"]
    return build_shared(units, OUT, link, hipcc(), HERE / ".build", verbose=verbose)


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv)
    print(p)
