"""FastAPI server: the OpenAI-compatible threaded chat API (/root/reference/server.py:89-631).

Routes (same paths, schemas and status codes as the reference):
  POST   /v1/threads/{thread_id}/chat/completions   threaded chat (history kept server-side), SSE or JSON
  POST   /v1/chat/completions                       stateless chat
  POST   /v1/agent/run                              stateless agent, SSE of raw agent events
  POST   /v1/threads/{thread_id}/agent/run          per-thread agent (thread profile, lazily-started sandbox), SSE
  POST   /v1/threads/{thread_id}/messages           append a message
  GET    /v1/threads/{thread_id}/messages           list messages (404 if the thread does not exist)
  POST   /v1/threads                                create a thread (optional system message / user / profile)
  DELETE /v1/threads/{thread_id}/messages           clear a thread (404 if missing)
  GET    /v1/models                                 models served by the engine
  GET    /health                                    liveness + engine state
  GET    /metrics                                   Prometheus metrics (new)

SSE behaviour (SURVEY.md §2.5.1/2.5.2, quirks Q1-Q3, Q6-Q8 fixed):
  * ``/chat/completions`` streams REAL tokens as the engine decodes them (the reference sliced the finished answer
    into 20-char frames after the whole agent run). Frames: a role frame, content frames, a stop frame with
    ``finish_reason``, an optional usage frame (``stream_options.include_usage``), ``data: [DONE]``. The stream stays
    OpenAI-SDK-safe: tool activity is NOT interleaved unless the client opts in with ``X-Kafka-Tool-Events: 1``
    (then ``{"type": "tool_result", ...}`` frames appear as in the reference). Errors: ``{"error": {...,
    "type": "server_error"}}`` then ``[DONE]``.
  * ``/agent/run`` streams every agent event as ``data: <json>`` then ``[DONE]``; errors use ``"agent_error"``.
  * threaded runs persist user/system messages first, then every assistant turn (with engine token ids) and tool
    result, under a per-thread lock; ``temperature=0`` means greedy (no ``or 0.7`` coercion); ``stop``, ``top_p``,
    penalties and ``seed`` reach the sampler; ``usage`` carries real token counts.
"""
from __future__ import annotations

import asyncio
import gc
import json
import os
import logging
import time
import uuid
from contextlib import asynccontextmanager
from typing import Any, AsyncGenerator, Optional

from fastapi import FastAPI, HTTPException, Request
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

from kafka_llm_service_amd.obs import trace
from kafka_llm_service_amd.kafka.types import (AgentRunRequest, ChatCompletionRequest, ChatMessage, Choice,
                                               ChatCompletionResponse, CreateThreadRequest, MessageContent, Usage)
from kafka_llm_service_amd.kafka.utils import convert_to_internal_message
from kafka_llm_service_amd.llm.types import Message
from kafka_llm_service_amd.obs import metrics as M
from kafka_llm_service_amd.server.state import ServerConfig, ServerState

log = logging.getLogger("kafka.server")

SSE_HEADERS = {"Cache-Control": "no-cache", "Connection": "keep-alive", "X-Accel-Buffering": "no"}


def _sse(obj: Any) -> str:
    return f"data: {json.dumps(obj, separators=(',', ':'))}\n\n"


def _chunk(cid: str, created: int, model: str, delta: dict, finish: Optional[str]) -> str:
    # compact JSON with explicit nulls, the shape Pydantic's model_dump_json gave the reference's frames
    d = {"role": delta.get("role"), "content": delta.get("content"), "tool_calls": delta.get("tool_calls")}
    return _sse({"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                 "choices": [{"index": 0, "delta": d, "finish_reason": finish}]})


async def _coalesce(gen: AsyncGenerator[str, None]) -> AsyncGenerator[str, None]:
    """Write every SSE frame that is ready in ONE transport send: a producer task drains ``gen`` into a queue and the
    response yields everything queued since the last write. A live token stream (one frame per engine step) is
    unchanged; bursts (usage + finish + [DONE], tool output, the stub provider's instant replies) stop costing one
    ASGI send each (~25 us of event-loop time per frame — the plumbing overhead SURVEY.md §6.2 measured)."""
    q: asyncio.Queue = asyncio.Queue()
    done = object()

    async def pump():
        try:
            async for frame in gen:
                q.put_nowait(frame)
        finally:
            q.put_nowait(done)

    task = asyncio.create_task(pump())
    try:
        while True:
            parts = [await q.get()]
            while not q.empty():
                parts.append(q.get_nowait())
            end = parts[-1] is done
            if end:
                parts.pop()
            if parts:
                yield "".join(parts)
            if end:
                break
        await task  # re-raise a producer failure
    finally:
        if not task.done():
            task.cancel()  # client went away: cancel the generation (engine abort runs in its finally blocks)


def _sampling_kwargs(req: ChatCompletionRequest) -> dict[str, Any]:
    kw: dict[str, Any] = {}
    if req.stop:
        kw["stop"] = [req.stop] if isinstance(req.stop, str) else list(req.stop)
    for k in ("top_p", "frequency_penalty", "presence_penalty", "seed", "user", "tool_choice"):
        v = getattr(req, k)
        if v is not None:
            kw[k] = v
    return kw


def create_app(config: ServerConfig | None = None, state: ServerState | None = None) -> FastAPI:
    st = state or ServerState(config or ServerConfig.from_env())

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        prof = None
        if os.environ.get("KAFKA_CPROFILE_SERVER"):  # host profile of the API process, dumped at shutdown
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        await st.start()
        # everything loaded so far (tokenizer tables, prompt sections, engine client, route closures: hundreds of
        # thousands of long-lived objects) leaves the cyclic GC's view: a full collection walking them stalled the
        # event loop for ~180 ms in the middle of a burst of new turns (profiles/r06/serve/: the loop-lag watchdog
        # caught the loop inside a collection's finalizers)
        gc.collect()
        gc.freeze()
        lag_task = None
        if trace.tracer() is not None:  # API event-loop lag (a blocked loop delays every request before its handler)
            lag_task = asyncio.get_running_loop().create_task(_loop_lag_monitor())
            _trace_gc(trace.tracer())
        try:
            yield
        finally:
            if lag_task is not None:
                lag_task.cancel()
            await st.stop()
            if prof is not None:
                import pstats

                prof.disable()
                with open(os.environ["KAFKA_CPROFILE_SERVER"], "w") as f:
                    ps = pstats.Stats(prof, stream=f)
                    ps.sort_stats("tottime").print_stats(45)
                    ps.sort_stats("cumtime").print_stats(60)

    def _trace_gc(tr) -> None:
        """Every cyclic-GC collection of this process as a `gc_gen<N>` span (a collection runs inside whatever
        allocation triggered it, so a stall dump shows only the allocating frame)."""
        t0 = [0.0]

        def cb(phase, info):
            if phase == "start":
                t0[0] = time.perf_counter()
            else:
                tr.complete(f"gc_gen{info.get('generation')}", "gc", t0[0], time.perf_counter(), "gc")
        gc.callbacks.append(cb)

    async def _loop_lag_monitor(period: float = 0.002) -> None:
        """Sleep `period` over and over; every wake-up later than 2 ms past its deadline is an `api_loop_lag` span
        (the time the event loop was busy elsewhere: a request arriving then waits that long before its handler)."""
        tr = trace.tracer()
        beat = [time.perf_counter()]
        dump = os.environ.get("KAFKA_LOOP_STALL_DUMP")
        if dump:  # diagnosis: a watchdog thread writes the loop thread's stack whenever it misses its beat by 50 ms
            import sys
            import threading
            import traceback

            loop_tid = threading.get_ident()

            def _watch():
                seen = 0.0
                with open(dump, "a") as f:
                    while True:
                        time.sleep(0.01)
                        b = beat[0]
                        if time.perf_counter() - b > 0.05 and b != seen:
                            seen = b
                            names = {t.ident: t.name for t in threading.enumerate()}
                            f.write(f"--- loop stalled {1e3 * (time.perf_counter() - b):.0f} ms\n")
                            for tid, fr in sys._current_frames().items():  # every thread: who holds the GIL?
                                if tid == threading.get_ident():
                                    continue
                                tag = "LOOP" if tid == loop_tid else names.get(tid, str(tid))
                                f.write(f"[{tag}]\n" + "".join(traceback.format_stack(fr)[-6:]))
                            f.flush()

            threading.Thread(target=_watch, daemon=True, name="loop-stall-dump").start()
        while True:
            t = time.perf_counter()
            await asyncio.sleep(period)
            beat[0] = time.perf_counter()
            late = beat[0] - t - period
            if late > 0.002:
                tr.complete("api_loop_lag", "api", t + period, t + period + late, "loop")

    app = FastAPI(title="kafka-llm-service-amd", lifespan=lifespan)
    app.state.kafka = st
    app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True, allow_methods=["*"],
                       allow_headers=["*"])

    def _require():
        if not st.ready:
            raise HTTPException(status_code=503, detail="Server not initialized")

    # ------------------------------------------------------------------------------------------------------------
    async def completion_events(messages: list[Message], req: ChatCompletionRequest, thread_id: str | None,
                                tool_events: bool) -> AsyncGenerator[str, None]:
        cid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        created = int(time.time())
        model = req.model
        t0 = time.perf_counter()
        first = True
        t_first = None
        finish = "stop"
        usage = None
        # content frames are the per-token hot path of the API loop (64 streams x ~110 tokens/s each): the constant
        # part of the frame is formatted once per request and only the text is JSON-encoded per token (the same
        # bytes as _chunk(..., {"content": text}, None))
        head = ('data: {"id":%s,"object":"chat.completion.chunk","created":%d,"model":%s,"choices":[{"index":0,'
                '"delta":{"role":null,"content":' % (json.dumps(cid), created, json.dumps(model)))
        tail = ',"tool_calls":null},"finish_reason":null}]}\n\n'
        try:
            yield _chunk(cid, created, model, {"role": "assistant"}, None)
            async for ev in st.run_agent(messages, req.model, req.temperature, req.max_tokens, thread_id,
                                         **_sampling_kwargs(req)):
                et = ev.get("type")
                if et == "tool_result":
                    if tool_events:
                        yield _sse({k: ev[k] for k in ("type", "tool_call_id", "tool_name", "delta", "is_complete")})
                    continue
                if et == "agent_done":
                    if ev.get("usage"):
                        usage = ev["usage"]
                    if ev.get("reason") == "max_iterations":
                        finish = "length"
                    continue
                ch = ev.get("choices")
                if not ch:
                    continue
                delta = ch[0].get("delta") or {}
                text = delta.get("content")
                if text:
                    if first:
                        t_first = time.perf_counter()
                        M.TTFT.observe(t_first - t0)
                        tr = trace.tracer()
                        if tr is not None:  # request in -> first content frame handed to the response
                            tr.complete("api_http_ttft", "api", t0, t_first, f"thr:{thread_id}")
                        first = False
                    yield head + json.dumps(text) + tail
                if ch[0].get("finish_reason") == "length":
                    finish = "length"
            end = _chunk(cid, created, model, {}, finish)
            if req.stream_options and req.stream_options.include_usage:
                u = usage or {}
                end += _sse({"id": cid, "object": "chat.completion.chunk", "created": created, "model": model,
                             "choices": [], "usage": {k: u.get(k, 0) for k in ("prompt_tokens", "completion_tokens",
                                                                              "total_tokens")}})
            tail_frames = end  # finish + usage + [DONE] leave in one send
        except Exception as e:  # the reference's error frame (server.py:375-377)
            log.exception("completion stream failed")
            tail_frames = _sse({"error": {"message": str(e), "type": "server_error"}})
        t_end = time.perf_counter()
        M.E2E.observe(t_end - t0)
        n_out = (usage or {}).get("completion_tokens", 0)
        if n_out:
            M.OUTPUT_TOKENS.inc(n_out)
            if n_out > 1 and t_first is not None:
                M.TPOT.observe((t_end - t_first) / (n_out - 1))
        yield tail_frames + "data: [DONE]\n\n"

    async def completion_json(messages, req: ChatCompletionRequest, thread_id: str | None) -> ChatCompletionResponse:
        content, usage, finish = "", {}, "stop"
        async for ev in st.run_agent(messages, req.model, req.temperature, req.max_tokens, thread_id,
                                     **_sampling_kwargs(req)):
            if ev.get("type") == "agent_done":
                content = ev.get("final_content") or ev.get("summary") or content
                usage = ev.get("usage") or usage
                if ev.get("reason") == "max_iterations":
                    finish = "length"
        return ChatCompletionResponse(
            id=f"chatcmpl-{uuid.uuid4().hex[:24]}", created=int(time.time()), model=req.model,
            choices=[Choice(message=MessageContent(content=content), finish_reason=finish)],
            usage=Usage(prompt_tokens=usage.get("prompt_tokens", 0), completion_tokens=usage.get("completion_tokens", 0),
                        total_tokens=usage.get("total_tokens", 0)))

    @app.post("/v1/threads/{thread_id}/chat/completions")
    async def thread_chat(thread_id: str, req: ChatCompletionRequest, request: Request):
        _require()
        M.REQUESTS.labels(route="thread_chat").inc()
        new = [convert_to_internal_message(m) for m in req.messages]
        tool_events = request.headers.get("x-kafka-tool-events") == "1"
        if req.stream:
            return StreamingResponse(_coalesce(completion_events(new, req, thread_id, tool_events)),
                                     media_type="text/event-stream", headers=SSE_HEADERS)
        return await completion_json(new, req, thread_id)

    @app.post("/v1/chat/completions")
    async def chat(req: ChatCompletionRequest, request: Request):
        _require()
        M.REQUESTS.labels(route="chat").inc()
        msgs = [convert_to_internal_message(m) for m in req.messages]
        tool_events = request.headers.get("x-kafka-tool-events") == "1"
        if req.stream:
            return StreamingResponse(_coalesce(completion_events(msgs, req, None, tool_events)),
                                     media_type="text/event-stream", headers=SSE_HEADERS)
        return await completion_json(msgs, req, None)

    async def agent_events(gen) -> AsyncGenerator[str, None]:
        # the agent routes feed the same serving metrics as the chat route: TTFT at the first generated frame
        # (content or a tool-call delta), end-to-end time, output tokens and TPOT from the run's summed usage
        t0 = time.perf_counter()
        t_first = None
        n_out = 0
        try:
            async for ev in gen:
                if t_first is None:
                    ch = ev.get("choices")
                    delta = (ch[0].get("delta") or {}) if ch else {}
                    if delta.get("content") or delta.get("tool_calls"):
                        t_first = time.perf_counter()
                        M.TTFT.observe(t_first - t0)
                if ev.get("type") == "agent_done":
                    n_out = (ev.get("usage") or {}).get("completion_tokens", 0) or 0
                yield f"data: {json.dumps(ev)}\n\n"  # json.dumps spacing, as the reference
        except Exception as e:
            log.exception("agent stream failed")
            yield f"data: {json.dumps({'error': {'message': str(e), 'type': 'agent_error'}})}\n\n"
        t_end = time.perf_counter()
        M.E2E.observe(t_end - t0)
        if n_out:
            M.OUTPUT_TOKENS.inc(n_out)
            if n_out > 1 and t_first is not None:
                M.TPOT.observe((t_end - t_first) / (n_out - 1))
        yield "data: [DONE]\n\n"

    @app.post("/v1/agent/run")
    async def agent_run(req: AgentRunRequest):
        _require()
        M.REQUESTS.labels(route="agent_run").inc()
        msgs = [convert_to_internal_message(m) for m in req.messages]
        return StreamingResponse(_coalesce(agent_events(st.run_agent(msgs, req.model, req.temperature, req.max_tokens,
                                                                     None))),
                                 media_type="text/event-stream", headers=SSE_HEADERS)

    @app.post("/v1/threads/{thread_id}/agent/run")
    async def thread_agent_run(thread_id: str, req: AgentRunRequest):
        _require()
        M.REQUESTS.labels(route="thread_agent_run").inc()
        if not await st.db.thread_exists(thread_id):
            await st.db.create_thread(thread_id=thread_id)
        msgs = [convert_to_internal_message(m) for m in req.messages]
        return StreamingResponse(_coalesce(agent_events(st.run_thread_agent(thread_id, msgs, req.model,
                                                                            req.temperature, req.max_tokens))),
                                 media_type="text/event-stream", headers=SSE_HEADERS)

    @app.post("/v1/threads/{thread_id}/messages")
    async def add_message(thread_id: str, message: ChatMessage):
        _require()
        if not await st.db.thread_exists(thread_id):
            await st.db.create_thread(thread_id=thread_id)
        mid = await st.db.add_message(thread_id, convert_to_internal_message(message))
        return {"success": True, "message_id": mid}

    @app.get("/v1/threads/{thread_id}/messages")
    async def get_messages(thread_id: str):
        _require()
        if not await st.db.thread_exists(thread_id):
            raise HTTPException(status_code=404, detail="Thread not found")
        msgs = await st.db.get_thread_messages(thread_id)
        return {"thread_id": thread_id, "messages": [m.to_dict() for m in msgs]}

    @app.post("/v1/threads")
    async def create_thread(req: Optional[CreateThreadRequest] = None):
        _require()
        req = req or CreateThreadRequest()
        t = await st.db.create_thread(system_message=req.system_message, user_id=req.user_id,
                                      kafka_profile_id=req.kafka_profile_id, metadata=req.metadata)
        return {"thread_id": t["id"], "created_at": t["created_at"]}

    @app.delete("/v1/threads/{thread_id}/messages")
    async def clear_thread(thread_id: str):
        _require()
        if not await st.db.thread_exists(thread_id):
            raise HTTPException(status_code=404, detail="Thread not found")
        return {"success": True, "deleted_count": await st.db.delete_thread_messages(thread_id)}

    @app.get("/v1/models")
    async def list_models():
        return {"object": "list", "data": [{"id": m, "object": "model", "owned_by": "kafka-llm-service-amd"}
                                           for m in st.model_ids()]}

    @app.get("/health")
    async def health():
        return {"status": "healthy", "kafka_initialized": st.ready, "engine": st.engine_health()}

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(M.render(st), media_type="text/plain; version=0.0.4")

    @app.exception_handler(ValueError)
    async def _value_error(request: Request, exc: ValueError):
        return JSONResponse({"detail": str(exc)}, status_code=400)

    from kafka_llm_service_amd.engine.client import EngineUnavailable

    @app.exception_handler(EngineUnavailable)
    async def _engine_unavailable(request: Request, exc: EngineUnavailable):
        # a dead / restarting replica (or an RCCL collective timeout that took its TP group down) is a transient
        # server condition: 503 so clients retry, the stream path reports it as an error frame
        return JSONResponse({"detail": str(exc)}, status_code=503)

    return app
