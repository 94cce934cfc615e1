"""Tokenizer, incremental detokenizer and chat templates for the Llama-3 / Mixtral engines.

No Llama-3 tokenizer can be downloaded here, so the engine ships its own deterministic
byte-level BPE, trained with the ``tokenizers`` library on a fixed in-repo corpus (``assets/bpe_corpus.txt``) and
stored as ``assets/kafka_bpe.json``. Its regular tokens take the low ids; the Llama-3 special tokens keep their real
ids (128000 ``<|begin_of_text|>`` ... 128009 ``<|eot_id|>``, 128010 ``<|python_tag|>``), so prompts have the exact
special-token structure and the model's 128256-row embedding is fully addressable. Ids between the trained vocabulary
and 128000 (which a random-init model samples freely) decode to deterministic pseudo-words, so streams show text.

If a real ``tokenizer.json`` is available (``KAFKA_TOKENIZER``), it is used instead.
"""
from __future__ import annotations

import json
import os
import threading
from functools import lru_cache
from pathlib import Path

ASSETS = Path(__file__).resolve().parent / "assets"

LLAMA3_SPECIAL = {
    "<|begin_of_text|>": 128000, "<|end_of_text|>": 128001, "<|start_header_id|>": 128006,
    "<|end_header_id|>": 128007, "<|eom_id|>": 128008, "<|eot_id|>": 128009, "<|python_tag|>": 128010,
}
MISTRAL_SPECIAL = {"<s>": 1, "</s>": 2, "[INST]": 3, "[/INST]": 4, "[TOOL_CALLS]": 5, "[AVAILABLE_TOOLS]": 6,
                   "[/AVAILABLE_TOOLS]": 7, "[TOOL_RESULTS]": 8, "[/TOOL_RESULTS]": 9}

_SYL = ["ka", "fu", "ro", "mi", "te", "sa", "no", "li", "pe", "du", "va", "zo", "ne", "qi", "bo", "ha"]


def pseudo_word(i: int) -> str:
    s = ""
    x = i
    for _ in range(2 + (i % 2)):
        s += _SYL[x % 16]
        x //= 16
    return " " + s


def _train(corpus: str, vocab_size: int):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    paras = [p for p in corpus.split("\n\n") if p.strip()]
    tok.train_from_iterator(paras, tr)
    return tok


_LOCK = threading.Lock()


def _load_base():
    from tokenizers import Tokenizer

    custom = os.environ.get("KAFKA_TOKENIZER")
    if custom:
        return Tokenizer.from_file(custom), True
    path = ASSETS / "kafka_bpe.json"
    with _LOCK:
        if not path.exists():
            corpus = (ASSETS / "bpe_corpus.txt").read_text(encoding="utf-8")
            tok = _train(corpus, 16000)
            tmp = path.with_suffix(".tmp")
            tok.save(str(tmp))
            os.replace(tmp, path)
    return Tokenizer.from_file(str(path)), False


class KafkaTokenizer:
    """family: "llama3" (vocab 128256) or "mistral" (vocab 32000)."""

    def __init__(self, family: str = "llama3", vocab_size: int = 128256):
        self.family = family
        self.vocab_size = vocab_size
        self.base, self.external = _load_base()
        self.n_base = self.base.get_vocab_size()
        if family == "llama3":
            self.special = dict(LLAMA3_SPECIAL)
            self.special_start = 128000
            self.offset = 0
            self.bos, self.eos_ids = 128000, [128001, 128008, 128009]
        else:
            self.special = dict(MISTRAL_SPECIAL)
            self.special_start = 0
            self.offset = 16  # regular tokens shifted past the control ids
            self.bos, self.eos_ids = 1, [2]
        self.id_to_special = {v: k for k, v in self.special.items()}

    # --- encode / decode --------------------------------------------------------------------------------------
    def encode(self, text: str) -> list[int]:
        if not text:
            return []
        ids = self.base.encode(text).ids
        return [i + self.offset for i in ids] if self.offset else ids

    def special_id(self, name: str) -> int:
        return self.special[name]

    def is_special(self, i: int) -> bool:
        return i in self.id_to_special or (self.family == "llama3" and i >= self.special_start)

    def _piece_ids(self, ids):
        """Split ids into runs: (kind, payload) with kind base / special / pseudo."""
        run: list[int] = []
        for i in ids:
            j = i - self.offset
            if i in self.id_to_special or (self.family == "llama3" and i >= self.special_start) or j < 0:
                if run:
                    yield "base", run
                    run = []
                yield "special", i
            elif j >= self.n_base:
                if run:
                    yield "base", run
                    run = []
                yield "pseudo", i
            else:
                run.append(j)
        if run:
            yield "base", run

    def decode(self, ids: list[int], skip_special_tokens: bool = True) -> str:
        out = []
        for kind, p in self._piece_ids(ids):
            if kind == "base":
                out.append(self.base.decode(p))
            elif kind == "pseudo":
                out.append(pseudo_word(p))
            elif not skip_special_tokens:
                out.append(self.id_to_special.get(p, f"<|reserved_{p}|>"))
        return "".join(out)


class IncrementalDetokenizer:
    """Streams text for a growing id list without re-decoding everything: decodes a short window and emits only
    text that is stable (a trailing U+FFFD means an incomplete UTF-8 byte sequence: wait for more tokens)."""

    def __init__(self, tok: KafkaTokenizer, skip_special_tokens: bool = True):
        self.tok = tok
        self.skip = skip_special_tokens
        self.ids: list[int] = []
        self.prefix_offset = 0
        self.read_offset = 0
        self.text = ""
        # the shipped byte-level BPE decodes a concatenation to the concatenation of the pieces' decodes whenever
        # no UTF-8 sequence is split, so a token following fully emitted text is decoded ALONE (one decode per
        # streamed token instead of two windows); an external tokenizer.json (e.g. SentencePiece spacing) keeps the
        # window diff
        self.byte_level = not getattr(tok, "external", True)

    def add(self, new_ids: list[int]) -> str:
        if self.byte_level and self.read_offset == len(self.ids):
            self.ids.extend(new_ids)
            piece = self.tok.decode(new_ids, self.skip)
            if not piece.endswith("\ufffd"):
                self.prefix_offset = self.read_offset = len(self.ids)
                self.text += piece
                return piece
        else:
            self.ids.extend(new_ids)
        prefix = self.tok.decode(self.ids[self.prefix_offset:self.read_offset], self.skip)
        full = self.tok.decode(self.ids[self.prefix_offset:], self.skip)
        if len(full) <= len(prefix) or full.endswith("\ufffd"):
            return ""
        delta = full[len(prefix):]
        self.prefix_offset = self.read_offset
        self.read_offset = len(self.ids)
        self.text += delta
        return delta


@lru_cache(maxsize=4)
def get_tokenizer(family: str = "llama3", vocab_size: int = 128256) -> KafkaTokenizer:
    return KafkaTokenizer(family, vocab_size)


def tokenizer_for_model(model_cfg) -> KafkaTokenizer:
    fam = "mistral" if model_cfg.arch == "mixtral" or model_cfg.vocab_size <= 32000 else "llama3"
    return get_tokenizer(fam, model_cfg.vocab_size)
