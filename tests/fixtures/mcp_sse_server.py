"""A legacy HTTP+SSE MCP server for tests (MCP 2024-11-05): GET /sse streams `endpoint` then `message` events,
POST /messages?session=<id> takes JSON-RPC. Streamable HTTP (POST /sse) is refused with 405, so a client must fall
back to SSE. Tools: echo / add (as tests/fixtures/mcp_echo_server.py). Usage: python mcp_sse_server.py PORT"""
import asyncio
import json
import sys
import uuid

import uvicorn
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse

TOOLS = [{"name": "echo", "description": "echo text", "inputSchema": {"type": "object", "properties": {
    "text": {"type": "string"}}, "required": ["text"]}},
         {"name": "add", "description": "add numbers", "inputSchema": {"type": "object", "properties": {
             "a": {"type": "number"}, "b": {"type": "number"}}}}]
app = FastAPI()
queues: dict[str, asyncio.Queue] = {}


def handle(msg):
    m = msg["method"]
    if m == "initialize":
        return {"protocolVersion": msg["params"]["protocolVersion"], "capabilities": {"tools": {}},
                "serverInfo": {"name": "sse-echo", "version": "0"}}
    if m == "tools/list":
        return {"tools": TOOLS}
    a = msg["params"]["arguments"]
    text = a["text"] if msg["params"]["name"] == "echo" else str(a["a"] + a["b"])
    return {"content": [{"type": "text", "text": text}]}


@app.get("/sse")
async def sse():
    sid = uuid.uuid4().hex
    q = queues[sid] = asyncio.Queue()

    async def gen():
        yield f"event: endpoint\ndata: /messages?session={sid}\n\n"
        while True:
            yield f"event: message\ndata: {json.dumps(await q.get())}\n\n"

    return StreamingResponse(gen(), media_type="text/event-stream")


@app.post("/sse")
async def no_streamable_http():
    return Response(status_code=405)


@app.post("/messages")
async def messages(request: Request, session: str):
    msg = await request.json()
    if "id" in msg:
        await queues[session].put({"jsonrpc": "2.0", "id": msg["id"], "result": handle(msg)})
    return JSONResponse({"ok": True}, status_code=202)


if __name__ == "__main__":
    uvicorn.run(app, host="127.0.0.1", port=int(sys.argv[1]), log_level="warning")
