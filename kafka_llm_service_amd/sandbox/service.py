"""The sandbox service: the HTTP endpoint that sandbox tools run against (``/health``, ``/claim``, ``/run``, ``/reset``).

The reference only ships the CLIENT side (/root/reference/src/sandbox/local.py, daytona.py) and relies on a service
running inside a Daytona VM. This is a local implementation of that service contract so the
shell / notebook tools work offline:
  * ``create_shell {shell_id}`` starts a persistent bash session; ``shell_exec {shell_id, command, timeout?}`` runs a
    command in it and streams stdout/stderr line by line, ending with the exit code,
  * ``notebook_run_cell {code, description?, timeout?}`` runs Python in one persistent interpreter (variables survive
    between cells) and streams its output,
  * ``/claim {"config": {...}}`` stores the thread environment, exported into every session started afterwards.
Run: ``python -m kafka_llm_service_amd.sandbox.service --port 8081 --workdir /tmp/sbx``.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import uuid
from typing import Any, AsyncGenerator

from contextlib import asynccontextmanager

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, StreamingResponse

_KERNEL_SRC = r'''
import sys, json, traceback, io, contextlib, ast
g = {"__name__": "__main__"}
out = sys.stdout
while True:
    line = sys.stdin.readline()
    if not line:
        break
    req = json.loads(line)
    marker = req["marker"]
    class W(io.TextIOBase):
        def write(self, s):
            if s:
                out.write(json.dumps({"o": s}) + "\n"); out.flush()
            return len(s)
    w = W()
    code = 0
    with contextlib.redirect_stdout(w), contextlib.redirect_stderr(w):
        try:
            tree = ast.parse(req["code"], "<cell>", "exec")
            last = tree.body.pop() if tree.body and isinstance(tree.body[-1], ast.Expr) else None
            exec(compile(tree, "<cell>", "exec"), g)
            if last is not None:  # like a notebook: show the value of a trailing expression
                val = eval(compile(ast.Expression(last.value), "<cell>", "eval"), g)
                if val is not None:
                    print(repr(val))
        except BaseException:
            traceback.print_exc()
            code = 1
    out.write(json.dumps({"done": marker, "exit_code": code}) + "\n"); out.flush()
'''


class ShellSession:
    def __init__(self, shell_id: str, cwd: str, env: dict[str, str]):
        self.shell_id = shell_id
        self.cwd = cwd
        self.env = env
        self.proc: asyncio.subprocess.Process | None = None
        self.lock = asyncio.Lock()

    async def start(self) -> None:
        self.proc = await asyncio.create_subprocess_exec(
            "bash", "--noprofile", "--norc", stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
            stderr=asyncio.subprocess.STDOUT, cwd=self.cwd, env=self.env)

    async def run(self, command: str, timeout: float) -> AsyncGenerator[dict, None]:
        async with self.lock:
            assert self.proc and self.proc.stdin and self.proc.stdout
            marker = f"__KAFKA_DONE_{uuid.uuid4().hex}__"
            self.proc.stdin.write(f"{{ {command}\n}} 2>&1; echo \"{marker}$?\"\n".encode())
            await self.proc.stdin.drain()
            loop = asyncio.get_running_loop()
            deadline = loop.time() + timeout
            while True:
                remaining = deadline - loop.time()
                if remaining <= 0:
                    self.proc.send_signal(2)
                    yield {"type": "error", "data": f"\n[timed out after {timeout:.0f}s]\n", "is_complete": True,
                           "exit_code": 124}
                    return
                try:
                    line = await asyncio.wait_for(self.proc.stdout.readline(), remaining)
                except asyncio.TimeoutError:
                    continue
                if not line:
                    yield {"type": "error", "data": "[shell exited]", "is_complete": True, "exit_code": -1}
                    return
                text = line.decode(errors="replace")
                if marker in text:
                    pre, _, code = text.partition(marker)
                    if pre:
                        yield {"type": "output", "data": pre}
                    yield {"type": "complete", "data": "", "is_complete": True,
                           "exit_code": int(code.strip() or 0)}
                    return
                yield {"type": "output", "data": text}

    async def close(self) -> None:
        if self.proc and self.proc.returncode is None:
            self.proc.kill()
            await self.proc.wait()


class PythonKernel:
    def __init__(self, cwd: str, env: dict[str, str]):
        self.cwd, self.env = cwd, env
        self.proc: asyncio.subprocess.Process | None = None
        self.lock = asyncio.Lock()

    async def ensure(self) -> None:
        if self.proc is None or self.proc.returncode is not None:
            self.proc = await asyncio.create_subprocess_exec(
                sys.executable, "-u", "-c", _KERNEL_SRC, stdin=asyncio.subprocess.PIPE,
                stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.STDOUT, cwd=self.cwd, env=self.env)

    async def run(self, code: str, timeout: float) -> AsyncGenerator[dict, None]:
        async with self.lock:
            await self.ensure()
            marker = uuid.uuid4().hex
            self.proc.stdin.write((json.dumps({"code": code, "marker": marker}) + "\n").encode())
            await self.proc.stdin.drain()
            loop = asyncio.get_running_loop()
            deadline = loop.time() + timeout
            while True:
                remaining = deadline - loop.time()
                if remaining <= 0:
                    self.proc.kill()
                    self.proc = None
                    yield {"type": "error", "data": f"\n[cell timed out after {timeout:.0f}s; kernel restarted]\n",
                           "is_complete": True, "exit_code": 124}
                    return
                try:
                    line = await asyncio.wait_for(self.proc.stdout.readline(), remaining)
                except asyncio.TimeoutError:
                    continue
                if not line:
                    self.proc = None
                    yield {"type": "error", "data": "[kernel died]", "is_complete": True, "exit_code": -1}
                    return
                try:
                    msg = json.loads(line)
                except json.JSONDecodeError:
                    yield {"type": "output", "data": line.decode(errors="replace")}
                    continue
                if msg.get("done") == marker:
                    yield {"type": "complete", "data": "", "is_complete": True, "exit_code": msg.get("exit_code", 0)}
                    return
                if "o" in msg:
                    yield {"type": "output", "data": msg["o"]}

    async def close(self) -> None:
        if self.proc and self.proc.returncode is None:
            self.proc.kill()
            await self.proc.wait()


class SandboxService:
    def __init__(self, workdir: str):
        self.workdir = os.path.abspath(workdir)
        os.makedirs(self.workdir, exist_ok=True)
        self.claimed = False
        self.env: dict[str, str] = dict(os.environ)
        self.shells: dict[str, ShellSession] = {}
        self.kernel: PythonKernel | None = None

    async def claim(self, config: dict[str, Any]) -> None:
        self.env.update({k: str(v) for k, v in (config or {}).items()})
        self.claimed = True

    async def reset(self) -> None:
        for s in self.shells.values():
            await s.close()
        self.shells.clear()
        if self.kernel:
            await self.kernel.close()
            self.kernel = None

    async def run(self, tool: str, args: dict[str, Any]) -> AsyncGenerator[dict, None]:
        if tool == "create_shell":
            sid = str(args.get("shell_id") or "main")
            if sid in self.shells:
                yield {"type": "complete", "data": f"Shell '{sid}' already exists.", "is_complete": True,
                       "exit_code": 0}
                return
            s = ShellSession(sid, self.workdir, self.env)
            await s.start()
            self.shells[sid] = s
            yield {"type": "complete", "data": f"Shell '{sid}' created.", "is_complete": True, "exit_code": 0}
        elif tool == "shell_exec":
            sid = str(args.get("shell_id") or "main")
            if sid not in self.shells:
                yield {"type": "error", "data": f"Shell '{sid}' does not exist. Call create_shell first.",
                       "is_complete": True, "exit_code": 1}
                return
            async for ev in self.shells[sid].run(str(args.get("command", "")), float(args.get("timeout", 600))):
                yield ev
        elif tool == "notebook_run_cell":
            if self.kernel is None:
                self.kernel = PythonKernel(self.workdir, self.env)
            async for ev in self.kernel.run(str(args.get("code", "")), float(args.get("timeout", 3600))):
                yield ev
        else:
            yield {"type": "error", "data": f"Unknown sandbox tool: {tool}", "is_complete": True, "exit_code": 127}


def create_app(workdir: str) -> FastAPI:
    svc = SandboxService(workdir)

    @asynccontextmanager
    async def lifespan(app):
        yield
        await svc.reset()

    app = FastAPI(title="kafka sandbox service", lifespan=lifespan)
    app.state.svc = svc

    @app.get("/health")
    async def health():
        return {"healthy": True, "claimed": svc.claimed, "shells": sorted(svc.shells)}

    @app.post("/claim")
    async def claim(req: Request):
        body = await req.json()
        await svc.claim(body.get("config", {}))
        return {"success": True, "claimed": True}

    @app.post("/reset")
    async def reset():
        await svc.reset()
        return {"success": True}

    @app.post("/run")
    async def run(req: Request):
        body = await req.json()
        tool = body.get("tool_name")
        if not tool:
            return JSONResponse({"detail": "tool_name required"}, status_code=422)

        async def gen():
            async for ev in svc.run(tool, body.get("arguments") or {}):
                yield f"data: {json.dumps(ev)}\n\n"
            yield "data: [DONE]\n\n"
        return StreamingResponse(gen(), media_type="text/event-stream",
                                 headers={"Cache-Control": "no-cache", "X-Accel-Buffering": "no"})

    return app


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8081)
    ap.add_argument("--workdir", default=os.path.join(os.getcwd(), "sandbox_workdir"))
    a = ap.parse_args()
    import uvicorn

    uvicorn.run(create_app(a.workdir), host=a.host, port=a.port, log_level="warning")


if __name__ == "__main__":
    main()
