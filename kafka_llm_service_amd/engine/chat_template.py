"""Chat templates (Llama-3.1 tool format, Mistral) rendered straight to token ids, and the tool-call parser.

Prefix stability is the design constraint: a thread's prompt for turn t+1 must begin with the
exact token ids of turn t's prompt + generated reply, or the per-thread KV prefix cache misses. So
  * every message is rendered to ids independently and the ids are concatenated (no cross-message BPE merges),
  * the system block (prompt + tool schemas, fixed order, compact JSON) is byte-identical across requests, so the
    ~18k-token Kafka prefix is shared by ALL threads,
  * an assistant message that carries the engine's own ``token_ids`` is re-emitted verbatim (no re-tokenisation).

Llama-3.1 layout:
  <|begin_of_text|><|start_header_id|>system<|end_header_id|>\\n\\n{system}\\n\\n{tools block}<|eot_id|>
  <|start_header_id|>user<|end_header_id|>\\n\\n{text}<|eot_id|>
  <|start_header_id|>assistant<|end_header_id|>\\n\\n{text | <|python_tag|>{"name": .., "parameters": ..}}<|eot_id|>
  <|start_header_id|>ipython<|end_header_id|>\\n\\n{tool result}<|eot_id|>
  <|start_header_id|>assistant<|end_header_id|>\\n\\n                       <- generation prompt
"""
from __future__ import annotations

import json
from collections import OrderedDict
import uuid
from typing import Any

from kafka_llm_service_amd.engine.tokenizer import KafkaTokenizer
from kafka_llm_service_amd.llm.types import Message

TOOLS_PREAMBLE = ("# Tools\n\nYou can call the functions below. To call one, reply with <|python_tag|> followed by a "
                  "JSON object {\"name\": <function name>, \"parameters\": <arguments object>} per line, and "
                  "nothing else.\n\n")


def _tools_block(tools: list[dict] | None) -> str:
    if not tools:
        return ""
    return TOOLS_PREAMBLE + "\n".join(json.dumps(t, separators=(",", ":")) for t in tools)


class ChatTemplate:
    def __init__(self, tok: KafkaTokenizer):
        self.tok = tok
        self.llama = tok.family == "llama3"
        self._enc_cache: OrderedDict[str, list[int]] = OrderedDict()

    def _encode_cached(self, text: str) -> list[int]:
        """BPE of the (system prompt + tool schemas) block, memoised: it is the same ~70k characters for every request
        of every thread, and re-encoding it would cost the API loop milliseconds per request."""
        ids = self._enc_cache.get(text)
        if ids is None:
            ids = self.tok.encode(text)
            self._enc_cache[text] = ids
            if len(self._enc_cache) > 64:
                self._enc_cache.popitem(last=False)
        else:
            self._enc_cache.move_to_end(text)
        return ids

    # --- llama 3 ----------------------------------------------------------------------------------------------
    def _hdr(self, role: str) -> list[int]:
        t = self.tok
        return [t.special_id("<|start_header_id|>")] + t.encode(role) + [t.special_id("<|end_header_id|>")] + \
            t.encode("\n\n")

    def _eot(self) -> int:
        return self.tok.special_id("<|eot_id|>" if self.llama else "</s>")

    def render_message(self, m: Message) -> list[int]:
        t = self.tok
        if not self.llama:
            return self._render_mistral(m)
        if m.role == "assistant":
            ids = self._hdr("assistant")
            if m.token_ids:
                body = list(m.token_ids)
                return ids + body + ([] if body and body[-1] in t.eos_ids else [self._eot()])
            if m.tool_calls:
                if m.content:
                    ids += t.encode(m.content)
                ids.append(t.special_id("<|python_tag|>"))
                calls = [json.dumps({"name": c["function"]["name"], "parameters": _args(c)}, separators=(",", ":"))
                         for c in m.tool_calls]
                ids += t.encode("\n".join(calls))
                return ids + [t.special_id("<|eom_id|>")]
            return ids + t.encode(m.content or "") + [self._eot()]
        role = "ipython" if m.role == "tool" else m.role
        return self._hdr(role) + t.encode(m.content or "") + [self._eot()]

    def _render_mistral(self, m: Message) -> list[int]:
        t = self.tok
        if m.role == "assistant":
            if m.token_ids:
                body = list(m.token_ids)
                return body + ([] if body and body[-1] in t.eos_ids else [t.special_id("</s>")])
            if m.tool_calls:
                calls = [{"name": c["function"]["name"], "arguments": _args(c)} for c in m.tool_calls]
                return [t.special_id("[TOOL_CALLS]")] + t.encode(json.dumps(calls, separators=(",", ":"))) + \
                    [t.special_id("</s>")]
            return t.encode(m.content or "") + [t.special_id("</s>")]
        if m.role == "tool":
            return [t.special_id("[TOOL_RESULTS]")] + t.encode(m.content or "") + [t.special_id("[/TOOL_RESULTS]")]
        return [t.special_id("[INST]")] + t.encode(m.content or "") + [t.special_id("[/INST]")]

    def render(self, messages: list[Message], tools: list[dict] | None = None,
               add_generation_prompt: bool = True) -> list[int]:
        t = self.tok
        ids = [t.bos]
        msgs = list(messages)
        if self.llama:
            system = ""
            if msgs and msgs[0].role == "system":
                system = msgs[0].content or ""
                msgs = msgs[1:]
            block = _tools_block(tools)
            if system or block:
                text = system + ("\n\n" + block if system and block else block)
                ids += self._hdr("system") + self._encode_cached(text) + [self._eot()]
            for m in msgs:
                ids += self.render_message(m)
            if add_generation_prompt:
                ids += self._hdr("assistant")
            return ids
        block = _tools_block(tools)
        if block:
            ids += [t.special_id("[AVAILABLE_TOOLS]")] + self._encode_cached(block) + \
                [t.special_id("[/AVAILABLE_TOOLS]")]
        for m in msgs:
            ids += self.render_message(m)
        return ids

    def generation_prefix(self) -> list[int]:
        return self._hdr("assistant") if self.llama else []

    def tool_call_start_ids(self) -> set[int]:
        return {self.tok.special_id("<|python_tag|>")} if self.llama else {self.tok.special_id("[TOOL_CALLS]")}


def _args(call: dict) -> Any:
    a = call["function"].get("arguments") or "{}"
    try:
        return json.loads(a) if isinstance(a, str) else a
    except json.JSONDecodeError:
        return {}


def parse_tool_calls(text: str) -> list[dict] | None:
    """Parse a generated tool-call body (one JSON object per line, Llama-3.1 ``{"name", "parameters"}`` or a Mistral
    JSON list of ``{"name", "arguments"}``) into OpenAI ``tool_calls``; None if it is not valid tool-call output."""
    s = text.strip()
    if not s:
        return None
    objs: list[dict] = []
    try:
        v = json.loads(s)
        objs = v if isinstance(v, list) else [v]
    except json.JSONDecodeError:
        for line in s.replace(";\n", "\n").split("\n"):
            line = line.strip().rstrip(";")
            if not line:
                continue
            try:
                objs.append(json.loads(line))
            except json.JSONDecodeError:
                return None
    calls = []
    for i, o in enumerate(objs):
        if not isinstance(o, dict) or "name" not in o:
            return None
        args = o.get("parameters", o.get("arguments", {}))
        calls.append({"index": i, "id": f"call_{uuid.uuid4().hex[:24]}", "type": "function",
                      "function": {"name": str(o["name"]),
                                   "arguments": args if isinstance(args, str) else json.dumps(args)}})
    return calls or None
