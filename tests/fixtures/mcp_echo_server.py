"""A tiny stdio MCP server for tests (JSON-RPC 2.0, newline-delimited): tools/list + tools/call of `echo` / `add`."""
import json
import sys

TOOLS = [{"name": "echo", "description": "echo text", "inputSchema": {"type": "object", "properties": {
    "text": {"type": "string"}}, "required": ["text"]}},
         {"name": "add", "description": "add numbers", "inputSchema": {"type": "object", "properties": {
             "a": {"type": "number"}, "b": {"type": "number"}}}}]

for line in sys.stdin:
    msg = json.loads(line)
    if "id" not in msg:
        continue
    m = msg["method"]
    if m == "initialize":
        res = {"protocolVersion": msg["params"]["protocolVersion"], "capabilities": {"tools": {}},
               "serverInfo": {"name": "echo", "version": "0"}}
    elif m == "tools/list":
        res = {"tools": TOOLS}
    elif m == "tools/call":
        a = msg["params"]["arguments"]
        if msg["params"]["name"] == "echo":
            res = {"content": [{"type": "text", "text": a["text"]}]}
        else:
            res = {"content": [{"type": "text", "text": str(a["a"] + a["b"])}]}
    else:
        sys.stdout.write(json.dumps({"jsonrpc": "2.0", "id": msg["id"], "error": {"code": -32601,
                                                                                 "message": "no method"}}) + "\n")
        sys.stdout.flush()
        continue
    sys.stdout.write(json.dumps({"jsonrpc": "2.0", "id": msg["id"], "result": res}) + "\n")
    sys.stdout.flush()
