"""In-tree native build driver (hipcc / g++), no setuptools, no hipify.

Every extension of the package is built by calling the compilers directly so that
  * HIP sources are compiled exactly as written for gfx950 (``--offload-arch=gfx950``),
  * the resulting ``.so`` lands inside the package tree (it travels with the repo snapshot to the GPU box),
  * rebuilds are incremental (object newer than its source and every header in the source dir).

Used by ``kafka_llm_service_amd/ops/build.py`` (HIP kernels + torch bindings) and
``kafka_llm_service_amd/runtime/build.py`` (C++ KV/prefix-cache core).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sysconfig
from dataclasses import dataclass, field
from pathlib import Path

ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = os.environ.get("KAFKA_GPU_ARCH", "gfx950")


def hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    return str(p) if p.exists() else (shutil.which("hipcc") or "hipcc")


def torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    root = Path(torch.__file__).parent
    incs = [str(p) for p in ce.include_paths()]
    return root, incs, int(torch._C._GLIBCXX_USE_CXX11_ABI)


@dataclass
class Unit:
    src: Path
    compiler: str
    flags: list[str] = field(default_factory=list)


def _stale(obj: Path, src: Path, deps: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_shared(units: list[Unit], out: Path, link_flags: list[str], linker: str, build_dir: Path,
                 jobs: int | None = None, verbose: bool = False) -> Path:
    build_dir.mkdir(parents=True, exist_ok=True)
    objs: list[Path] = []
    todo: list[list[str]] = []
    for u in units:
        obj = build_dir / (u.src.name + ".o")
        objs.append(obj)
        deps = [p for p in u.src.parent.glob("*.h")]
        if _stale(obj, u.src, deps):
            todo.append([u.compiler, *u.flags, "-c", str(u.src), "-o", str(obj)])
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=min(jobs, len(todo))) as ex:
            for cmd, _ in zip(todo, ex.map(_run, todo)):
                if verbose:
                    print(" ".join(cmd))
    if todo or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        tmp = out.with_suffix(".so.tmp")
        _run([linker, "-shared", "-o", str(tmp), *[str(o) for o in objs], *link_flags])
        os.replace(tmp, out)
    return out


def python_include() -> str:
    return sysconfig.get_paths()["include"]
