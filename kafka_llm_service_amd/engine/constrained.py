"""Schema-constrained tool-call decoding (random-init models never emit a valid tool call, so the
agent / tool-calling configurations force well-formed calls with logit masks in the sampler).

A ``ToolCallConstraint`` is a per-request ``SamplingParams.allowed_tokens_fn``: before every sampled token the model
runner asks it for the allowed set (``None`` = unconstrained, a list of ids, or a cached boolean vocab mask) and masks
the other logits to -inf. The constraint is a small program (a Python generator) that walks the chat template's tool
call grammar token by token:

    llama3:  <|python_tag|> {"name":"<tool>","parameters":<object per the tool's JSON schema>} <|eom_id|>
    mistral: [TOOL_CALLS] [{"name":"<tool>","arguments":<object>}] </s>

* fixed JSON punctuation / keys are FORCED (one allowed id), tokenized segment by segment — byte-level BPE decodes a
  concatenation of separately encoded segments to the concatenated text, so the result is exactly
  ``json.dumps(..., separators=(",", ":"))`` shaped;
* the tool name and ``enum`` values are CHOICES over the tokenizations of the alternatives (a trie walk);
* free values are bounded: strings take "string-safe" tokens (no ``"``, ``\\`` or control bytes, checked on the token's
  bytes) and may close after >= 1 token, integers / numbers are one digit-only token (no leading zero), booleans are
  a choice, arrays hold one item, nested objects emit their required properties.
The model's own probabilities still pick among the allowed tokens (temperature / top-p apply), so with real weights
the constraint only removes malformed continuations. ``tool_choice``: ``"auto"`` lets the first token decide (the
constraint engages only once the model opens a tool call), ``"required"`` forces a call to any tool, a named function
forces that tool, ``"none"`` forbids the tool-call token.
"""
from __future__ import annotations

import json
from functools import lru_cache
from typing import Any, Iterator

import numpy as np

from kafka_llm_service_amd.engine.tokenizer import KafkaTokenizer

MAX_STR_TOKENS = 12


@lru_cache(maxsize=1)
def _byte_decoder() -> dict[str, int]:
    """Inverse of the GPT-2 byte-level alphabet used by the byte-level BPE (unicode char -> byte)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


class VocabClasses:
    """Boolean masks over the vocabulary, computed once per tokenizer."""

    def __init__(self, tok: KafkaTokenizer):
        V = tok.vocab_size
        dec = _byte_decoder()
        self.str_safe = np.zeros(V, dtype=bool)
        self.digits = np.zeros(V, dtype=bool)
        self.digits_nz = np.zeros(V, dtype=bool)  # digit-only tokens not starting with '0'
        for j in range(tok.n_base):
            piece = tok.base.id_to_token(j)
            if piece is None:
                continue
            try:
                bs = bytes(dec[c] for c in piece)
            except KeyError:
                continue
            i = j + tok.offset
            if i >= V or tok.is_special(i):
                continue
            if bs and all(b >= 0x20 and b not in (0x22, 0x5C, 0x7F) for b in bs):
                self.str_safe[i] = True
            if bs and all(0x30 <= b <= 0x39 for b in bs):
                self.digits[i] = True
                self.digits_nz[i] = bs[0] != 0x30
        # unused ids above the trained vocabulary decode to pseudo words (letters + a space): string-safe
        for i in range(tok.n_base + tok.offset, V):
            if not tok.is_special(i):
                self.str_safe[i] = True
        self._ranges: dict = {}

    def digit_range(self, tok: KafkaTokenizer, lo, hi) -> np.ndarray:
        """Mask of single digit-run tokens (no leading zero, or "0") whose integer value lies in [lo, hi]."""
        key = (lo, hi)
        m = self._ranges.get(key)
        if m is None:
            m = np.zeros(tok.vocab_size, dtype=bool)
            zero = tok.encode("0")[:1]
            for i in list(np.flatnonzero(self.digits_nz)) + zero:
                v = int(tok.decode([int(i)]))
                if (lo is None or v >= lo) and (hi is None or v <= hi):
                    m[i] = True
            self._ranges[key] = m
        return m


_CLASSES: dict[int, VocabClasses] = {}


def vocab_classes(tok: KafkaTokenizer) -> VocabClasses:
    c = _CLASSES.get(id(tok))
    if c is None:
        c = _CLASSES[id(tok)] = VocabClasses(tok)
    return c


class Mask:
    """An allowed set given as a cached vocab mask plus a few extra ids (cache key lets the runner reuse the device
    copy of the base mask)."""
    __slots__ = ("key", "base", "extra")

    def __init__(self, key: str, base: np.ndarray, extra: list[int]):
        self.key, self.base, self.extra = key, base, extra


class ToolCallConstraint:
    def __init__(self, tok: KafkaTokenizer, tools: list[dict], tool_choice: Any = "auto"):
        self.tok = tok
        self.cls = vocab_classes(tok)
        self.llama = tok.family == "llama3"
        self.start = tok.special_id("<|python_tag|>") if self.llama else tok.special_id("[TOOL_CALLS]")
        self.end = tok.special_id("<|eom_id|>") if self.llama else tok.eos_ids[0]
        self.tools = {t["function"]["name"]: t["function"].get("parameters") or {} for t in tools
                      if t.get("type", "function") == "function" and "function" in t}
        self.mode, names = self._mode(tool_choice)
        self.names = names
        self._gen: Iterator | None = None
        self._spec: Any = None
        self._n = 0
        self.done = False
        self._guards: list[tuple[int, frozenset]] = []  # (slot, E): speculated "output_ids[slot] not in E"
        # slot n -> guarded slot n - 1 when the spec LAUNCHED for slot n (the last __call__ for it: the runner asks at
        # launch) was speculated past the pending token n - 1; guard slots whose landed token broke the guess
        self._spec_from: dict[int, int] = {}
        self._violated: set[int] = set()

    def _mode(self, tc):
        if isinstance(tc, dict):
            name = (tc.get("function") or {}).get("name")
            if name not in self.tools:
                raise ValueError(f"tool_choice names an unknown tool: {name}")
            return "forced", [name]
        if tc in (None, "auto"):
            return "auto", list(self.tools)
        if tc == "required":
            return "forced", list(self.tools)
        if tc == "none":
            return "none", []
        raise ValueError(f"unsupported tool_choice: {tc!r}")

    # ---- runner protocol ----------------------------------------------------------------------------------------
    # ``output_ids`` may end with ONE placeholder (< 0): the token being sampled by the step in flight (the engine
    # plans step n+1 before step n's token lands). When the spec that token was drawn under makes the NEXT state
    # depend only on whether the token falls in a small set E — a Mask (free string: E = the closing quote; digits
    # and "none": E is empty, every token ends the value / the state) or the first free token of "auto" (E = the
    # tool-call start) — the program consumes a representative token outside E now and records the guard (slot, E).
    # When the real token lands inside E the guess was wrong: the program is rebuilt from the landed tokens, the guard
    # slot is remembered as violated (``plan_state`` keeps the row out of plans until then), and the token sampled
    # under the mis-predicted mask (slot + 1) is rolled back by the engine at its landing (``rollback_at``) — only if
    # the spec LAUNCHED for slot + 1 was the speculated one (a plan dropped and redone after the landing used the
    # real token). Choice states (tool names, enums, booleans: the next state depends on WHICH token) cannot be
    # predicted: ``plan_state`` -> "wait".
    def _advance(self, t: int) -> None:
        self._n += 1
        if self._spec is _FREE_FOREVER:
            return
        try:
            self._spec = self._gen.send(t)
        except StopIteration:
            self._spec = _FREE_FOREVER
            self.done = True

    def _enc(self, text: str) -> list[int]:
        """Token ids of a grammar segment, cached per tokenizer (the same keys / names / punctuation every call)."""
        cache = self.tok.__dict__.setdefault("_grammar_enc", {})
        ids = cache.get(text)
        if ids is None:
            ids = cache[text] = self.tok.encode(text)
        return ids

    def _start(self) -> None:
        if self._gen is None:
            self._gen = self._program()
            self._spec = next(self._gen)

    def _class_of(self, spec):
        """(representative token, E) for a spec whose successor state depends only on membership in E, else None."""
        if spec is _FREE_FOREVER:
            return 0, frozenset()
        if spec is None:  # "auto" before the first token: only the tool-call start token changes the state
            return (0 if self.start != 0 else 1), frozenset([self.start])
        if isinstance(spec, Mask):
            # digit masks end the value whichever token lands (a lone "0" included): nothing to guard
            extra = frozenset() if spec.key.startswith("digits") else frozenset(int(e) for e in spec.extra)
            k = (id(spec.base), spec.key, extra)
            rep = _REPS.get(k)
            if rep is None:
                cand = np.flatnonzero(spec.base[:4096]) if spec.base[:4096].any() else np.flatnonzero(spec.base)
                rep = _REPS[k] = next((int(c) for c in cand[:64] if int(c) not in extra), -1)
            return (rep, extra) if rep >= 0 else None
        return None

    def _validate(self, output_ids: list[int]) -> int | None:
        """Check every guard whose token has landed; on a violation rebuild the program from the landed tokens and
        return the guarded slot (the token after it was drawn under a wrong mask)."""
        bad = None
        keep = []
        for slot, extra in self._guards:
            t = output_ids[slot] if slot < len(output_ids) else -1
            if t < 0:
                keep.append((slot, extra))
            elif t in extra and bad is None:
                bad = slot
        self._guards = keep
        if bad is None:
            return None
        self._violated.add(bad)
        self._gen, self._spec, self._n, self.done, self._guards = None, None, 0, False, []
        self._start()
        for t in output_ids[:bad + 1]:
            self._advance(t)
        return bad

    def __call__(self, output_ids: list[int]):
        self._start()
        self._validate(output_ids)
        n = len(output_ids)
        spec_past = None
        while self._n < len(output_ids):
            t = output_ids[self._n]
            if t < 0:  # the in-flight token: speculate past it (plan_state said the spec allows it)
                if self._n != len(output_ids) - 1:
                    raise RuntimeError("constraint: only the last token may be pending")
                cls = self._class_of(self._spec)
                if cls is None:
                    raise RuntimeError("constraint: cannot plan past a pending token drawn from a choice")
                rep, extra = cls
                if extra:
                    self._guards.append((self._n, extra))
                    spec_past = self._n
                t = rep
            self._advance(t)
        if spec_past is not None:
            self._spec_from[n] = spec_past
        else:
            self._spec_from.pop(n, None)
        return None if self._spec is _FREE_FOREVER else self._spec

    def plan_state(self, output_ids: list[int]) -> str:
        """Can the row be planned while its last token is pending? "ok" | "wait" (choice state: sit this step
        out) | "rollback" (a landed token broke a guess: the pending token was drawn under a wrong mask)."""
        self._start()
        if self._validate(output_ids) is not None:
            return "rollback"
        n = len(output_ids)
        if n and output_ids[-1] < 0 and self._spec_from.get(n - 1) in self._violated:
            return "rollback"  # the pending token was drawn under a wrong guess: wait for its landing (rollback_at)
        if not output_ids or output_ids[-1] >= 0:
            return "ok"
        if self._n < len(output_ids) - 1:  # consume the landed tokens first (no speculation involved)
            self.__call__(output_ids[:-1])
        return "ok" if self._n >= len(output_ids) or self._class_of(self._spec) is not None else "wait"

    def rollback_at(self, output_ids: list[int], slot: int) -> bool:
        """At the landing of ``output_ids[slot]``: True if it was drawn under a mis-predicted mask (the token before
        it broke its guard) and must be discarded; the program is rebuilt from the landed tokens then."""
        self._validate(output_ids[:slot])
        g = self._spec_from.pop(slot, None)
        hit = g is not None and g in self._violated
        self._violated = {v for v in self._violated if v >= slot}
        return hit

    # ---- grammar -------------------------------------------------------------------------------------------------
    def _program(self):
        if self.mode == "none":
            m = np.ones(self.tok.vocab_size, dtype=bool)
            m[self.start] = False
            yield Mask("no_tool_start", m, [])
            return
        if self.mode == "auto":
            first = yield None
            if first != self.start:
                return
        else:
            yield [self.start]
        yield from self._forced('[{"name":"' if not self.llama else '{"name":"')
        name = yield from self._choice([n + '"' for n in self.names])
        name = name[:-1]
        yield from self._forced(',"parameters":' if self.llama else ',"arguments":')
        yield from self._value(self.tools.get(name) or {"type": "object"})
        yield from self._forced("}" if self.llama else "}]")
        yield [self.end]
        self.done = True

    def _forced(self, text: str):
        for i in self._enc(text):
            yield [i]

    def _choice(self, alts: list[str]):
        """Trie walk over the tokenizations of ``alts``; returns the chosen alternative."""
        seqs = [(a, self._enc(a)) for a in alts]
        pos = 0
        while True:
            live = [(a, s) for a, s in seqs if len(s) > pos]
            t = yield sorted({s[pos] for _, s in live})
            seqs = [(a, s) for a, s in live if s[pos] == t]
            pos += 1
            done = [a for a, s in seqs if len(s) == pos]
            if done:
                return done[0]

    def _value(self, schema: dict):
        """Emit one JSON value for ``schema`` (every value is self-delimiting, so no look-ahead is needed)."""
        if "enum" in schema and schema["enum"]:
            yield from self._choice([json.dumps(v, separators=(",", ":")) for v in schema["enum"]])
            return
        typ = schema.get("type", "string")
        if isinstance(typ, list):
            typ = next((t for t in typ if t != "null"), "string")
        if typ == "object":
            props = schema.get("properties") or {}
            req = [k for k in (schema.get("required") or []) if k in props]
            yield from self._forced("{")
            for j, k in enumerate(req):
                if j:
                    yield from self._forced(",")
                yield from self._forced(json.dumps(k) + ":")
                yield from self._value(props[k])
            yield from self._forced("}")
        elif typ == "array":
            # one item (the minimal non-empty array; enough for a well-formed call)
            yield from self._forced("[")
            yield from self._value(schema.get("items") or {"type": "string"})
            yield from self._forced("]")
        elif typ in ("integer", "number"):
            # one digit-only token without a leading zero (BPE digit runs cover 1..3 digits), or a lone "0";
            # "minimum" / "maximum" restrict the choice to tokens whose value is in range
            lo, hi = schema.get("minimum"), schema.get("maximum")
            if lo is None and hi is None:
                yield Mask("digits_nz", self.cls.digits_nz, self._enc("0")[:1])
                return
            m = self.cls.digit_range(self.tok, lo, hi)
            if m.any():
                yield Mask(f"digits[{lo},{hi}]", m, [])
            else:  # nothing representable in one token (e.g. a negative range): emit the bound itself
                yield from self._forced(json.dumps(lo if lo is not None else hi))
        elif typ == "boolean":
            yield from self._choice(["true", "false"])
        elif typ == "null":
            yield from self._forced("null")
        else:  # string (and anything unrecognised): 1..MAX_STR_TOKENS string-safe tokens, then the closing quote
            q = self._enc('"')
            yield from self._forced('"')
            yield Mask("str", self.cls.str_safe, [])
            for _ in range(MAX_STR_TOKENS - 1):
                t = yield Mask("str", self.cls.str_safe, q[:1])
                if t == q[0]:
                    for i in q[1:]:
                        yield [i]
                    return
            yield from self._forced('"')


_FREE_FOREVER = object()
_REPS: dict = {}  # (id(mask base), key, extras) -> a representative token outside the extras
