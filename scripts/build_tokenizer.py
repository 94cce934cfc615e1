#!/usr/bin/env python3
"""Train the engine's offline byte-level BPE tokenizers (``engine/assets/kafka_bpe_{llama3,mistral}.json.gz``).

No Llama-3 / Mistral tokenizer can be downloaded here, so the engine ships its own: a byte-level BPE with the
Llama-3 pre-tokenizer split (the public regex of the tiktoken-style Llama-3 tokenizer: contractions, letter runs with
one leading non-letter, 1-3 digit groups, punctuation runs, newline runs) trained on LOCAL text that is NOT the
reference's prompt (VERDICT r03 "Next round" #4):

* Python 3.10 stdlib docstrings and comments (``/usr/lib/python3.10``),
* docstrings and comments of the installed site-packages (transformers, torch, pandas, ... — English API prose),
* ``.md`` / ``.rst`` / ``.txt`` documentation under ``/usr`` and ``/opt/rocm`` (READMEs, licences, guides),
* ``/usr/share/doc`` (gzipped changelogs / copyright files) and man pages,
* a slice of raw Python source (code and JSON-like literals appear in tool schemas and tool results).

Everything is collected in sorted path order with fixed byte caps, so a rebuild on the same image reproduces the
corpus (its sha256 is recorded in the manifest). Vocabularies: llama3 = 128,000 regular ids (the Llama-3 special
tokens keep their real ids 128000..128255 on top, so the model's 128,256-row embedding is exactly the tokenizer's
id space); mistral = 31,984 regular ids (shifted past 16 control ids, 32,000 in total).

Usage: python scripts/build_tokenizer.py [--mb 160] [--out kafka_llm_service_amd/engine/assets]
"""
from __future__ import annotations

import argparse
import ast
import gzip
import hashlib
import io
import json
import os
import re
import sys
import time
import tokenize
from pathlib import Path

LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|"
                r"\s*[\r\n]+|\s+(?!\S)|\s+")
EXCLUDE = ("/root/reference", "/root/repo", "/proc", "/sys", "/tmp")


def _files(root: str, exts: tuple[str, ...], max_size: int = 4 << 20) -> list[str]:
    out = []
    for dp, dns, fns in os.walk(root):
        dns.sort()
        if dp.startswith(EXCLUDE) or "/.git" in dp or "__pycache__" in dp:
            dns[:] = []
            continue
        for f in sorted(fns):
            if f.endswith(exts):
                p = os.path.join(dp, f)
                try:
                    if os.path.isfile(p) and not os.path.islink(p) and 0 < os.path.getsize(p) <= max_size:
                        out.append(p)
                except OSError:
                    pass
    return out


def _py_prose(src: str) -> str:
    """Docstrings + comments of a Python file (the English prose of the API docs)."""
    parts = []
    try:
        tree = ast.parse(src)
        for node in ast.walk(tree):
            if isinstance(node, (ast.Module, ast.ClassDef, ast.FunctionDef, ast.AsyncFunctionDef)):
                d = ast.get_docstring(node, clean=True)
                if d and len(d) > 40:
                    parts.append(d)
    except (SyntaxError, ValueError, RecursionError, MemoryError):
        pass
    try:
        comments = []
        for tok in tokenize.generate_tokens(io.StringIO(src).readline):
            if tok.type == tokenize.COMMENT:
                c = tok.string.lstrip("#").strip()
                if len(c) > 20 and not c.startswith(("!", "-*-", "type:", "noqa", "pragma")):
                    comments.append(c)
        if comments:
            parts.append("\n".join(comments))
    except (tokenize.TokenError, IndentationError, SyntaxError):
        pass
    return "\n\n".join(parts)


_ROFF = re.compile(r"^\.[A-Za-z]{1,3}\b ?|\\f[BIRP]|\\-|\\\(.{2}|\\&|\\e", re.M)


def _read(p: str) -> str:
    try:
        raw = gzip.open(p).read() if p.endswith(".gz") else open(p, "rb").read()
    except (OSError, EOFError):
        return ""
    if b"\x00" in raw[:4096]:
        return ""
    try:
        return raw.decode("utf-8")
    except UnicodeDecodeError:
        return ""


def collect(total_mb: int, log=print) -> tuple[list[str], dict]:
    """Returns (paragraph list, manifest)."""
    budget = total_mb << 20
    # (name, share of the budget, iterator of texts)
    site = "/usr/local/lib/python3.10/dist-packages"

    def stdlib_prose():
        for p in _files("/usr/lib/python3.10", (".py",)):
            yield _py_prose(_read(p))

    def site_prose():
        # at most ~4 MB of prose per top-level package (sorted), so the corpus spans many projects' English
        per_pkg = 4 << 20
        for pkg in sorted(os.listdir(site)):
            root = os.path.join(site, pkg)
            if not os.path.isdir(root) or pkg.endswith((".dist-info", ".egg-info")) or pkg.startswith(("_", ".")):
                continue
            got = 0
            for p in _files(root, (".py",)):
                t = _py_prose(_read(p))
                got += len(t)
                yield t
                if got >= per_pkg:
                    break

    def docs():
        for root in ("/usr/share", "/usr/lib", "/opt/rocm", site, "/usr/local/share"):
            if os.path.isdir(root):
                for p in _files(root, (".md", ".rst", ".txt", ".markdown")):
                    if "LICENSE" in p.upper() or "COPYING" in p.upper():
                        continue  # near-duplicate licence texts would dominate the merges
                    yield _read(p)

    def share_doc():
        for p in _files("/usr/share/doc", (".gz", "README", "NEWS", "changelog")):
            if "copyright" in p:
                continue
            yield _read(p)
        for p in _files("/usr/share/man", (".gz",)):
            yield _ROFF.sub("", _read(p))

    def code():
        for p in _files("/usr/lib/python3.10", (".py",)):
            yield _read(p)

    sources = [("stdlib_prose", 0.20, stdlib_prose), ("site_prose", 0.40, site_prose), ("docs", 0.22, docs),
               ("share_doc", 0.03, share_doc), ("code", 0.15, code)]
    paras: list[str] = []
    manifest = {"sources": {}, "total_mb_cap": total_mb}
    h = hashlib.sha256()
    for name, share, gen in sources:
        cap, got, nfiles = int(budget * share), 0, 0
        t0 = time.time()
        for text in gen():
            if not text:
                continue
            for para in text.split("\n\n"):
                para = para.strip("\n")
                if len(para) < 8:
                    continue
                paras.append(para)
                b = para.encode("utf-8", "replace")
                h.update(b)
                got += len(b)
            nfiles += 1
            if got >= cap:
                break
        manifest["sources"][name] = {"bytes": got, "files": nfiles}
        log(f"  {name}: {got / 1e6:.1f} MB from {nfiles} files ({time.time() - t0:.0f} s)")
    manifest["corpus_sha256"] = h.hexdigest()
    manifest["paragraphs"] = len(paras)
    return paras, manifest


def train(paras: list[str], vocab_size: int):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(paras, tr, length=len(paras))
    return tok


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=160)
    ap.add_argument("--out", default=str(Path(__file__).resolve().parents[1] / "kafka_llm_service_amd/engine/assets"))
    ap.add_argument("--only", default="llama3,mistral")
    a = ap.parse_args()
    out = Path(a.out)
    t0 = time.time()
    print("collecting corpus ...", flush=True)
    paras, manifest = collect(a.mb)
    for fam, vs in (("llama3", 128000), ("mistral", 31984)):
        if fam not in a.only.split(","):
            continue
        t1 = time.time()
        tok = train(paras, vs)
        js = tok.to_str()
        with gzip.GzipFile(out / f"kafka_bpe_{fam}.json.gz", "wb", mtime=0) as f:
            f.write(js.encode("utf-8"))
        manifest[fam] = {"vocab_size": tok.get_vocab_size(), "merges": len(json.loads(js)["model"]["merges"]),
                         "train_s": round(time.time() - t1, 1)}
        print(f"{fam}: vocab {tok.get_vocab_size()} ({time.time() - t1:.0f} s)", flush=True)
    manifest["split_regex"] = LLAMA3_SPLIT
    (out / "kafka_bpe_manifest.json").write_text(json.dumps(manifest, indent=1) + "\n")
    print(f"done in {time.time() - t0:.0f} s", file=sys.stderr)


if __name__ == "__main__":
    main()
