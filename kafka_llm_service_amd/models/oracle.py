"""Correctness oracle: a dense, cache-free PyTorch forward of the same model.

Used by the engine integration tests: greedy output of the paged + prefix-cached + continuously-batched engine must
match re-running the whole sequence through this plain implementation at every step. ``fp32=True`` runs every
activation and every matmul in fp32 (weights upcast), the reference the engine's composed bf16 error is bounded
against (tests/test_numerics_gpu.py, smoke()).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from kafka_llm_service_amd.models.llama import TransformerLM
from kafka_llm_service_amd.models.moe import route


def _rms(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def _lin(x, w):
    """x @ w^T in x's dtype (fp32 activations upcast the bf16 weight)."""
    return F.linear(x, w if w.dtype == x.dtype else w.to(x.dtype))


def _rope(x, cs):  # x [T, H, D], cs [T, D]
    half = x.shape[-1] // 2
    c, s = cs[:, None, :half], cs[:, None, half:]
    x1, x2 = x[..., :half].float(), x[..., half:].float()
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).to(x.dtype)


@torch.inference_mode()
def dense_logits(model: TransformerLM, tokens: list[int], fp32: bool = False) -> torch.Tensor:
    """Logits [T, V] (fp32) for every position of ``tokens`` (TP=1 models only); ``fp32``: fp32 activations."""
    assert model.tp == 1
    cfg = model.cfg
    dev = model.device
    t = torch.tensor(tokens, device=dev)
    T = t.shape[0]
    pos = torch.arange(T, device=dev)
    cs = model.cos_sin[pos].float()
    h = F.embedding(t, model.embed)
    if fp32:
        h = h.float()
    D, hq, hkv = model.D, model.hq, model.hkv
    G = hq // hkv
    mask = torch.ones(T, T, dtype=torch.bool, device=dev).tril()
    for lw in model.layers:
        x = _rms(h, lw.input_norm, cfg.rms_norm_eps)
        qkv = _lin(x, lw.qkv)
        q = qkv[:, :hq * D].view(T, hq, D)
        k = qkv[:, hq * D:(hq + hkv) * D].view(T, hkv, D)
        v = qkv[:, (hq + hkv) * D:].view(T, hkv, D)
        q, k = _rope(q, cs), _rope(k, cs)
        kf = k.float().repeat_interleave(G, 1)
        vf = v.float().repeat_interleave(G, 1)
        s = torch.einsum("thd,shd->hts", q.float(), kf) * model.scale
        s = s.masked_fill(~mask[None], float("-inf"))
        o = torch.einsum("hts,shd->thd", torch.softmax(s, -1), vf).to(h.dtype)
        h = (h.float() + _lin(o.reshape(T, -1), lw.o).float()).to(h.dtype)
        x = _rms(h, lw.post_norm, cfg.rms_norm_eps)
        if lw.router is not None:
            w, e = route(_lin(x, lw.router), cfg.num_experts_per_tok)
            out = torch.zeros(T, x.shape[1], dtype=torch.float32, device=dev)
            for j in range(cfg.num_experts):
                sel = (e == j)
                rows = sel.any(-1).nonzero().flatten()
                if rows.numel() == 0:
                    continue
                gu = _lin(x[rows], lw.w13[j])
                Fh = gu.shape[-1] // 2
                a = (F.silu(gu[:, :Fh].float()) * gu[:, Fh:].float()).to(x.dtype)
                y = _lin(a, lw.w2[j]).float()
                out[rows] += y * (w * sel)[rows].sum(-1, keepdim=True)
            delta = out.to(h.dtype)
        else:
            gu = _lin(x, lw.gate_up)
            Fh = gu.shape[-1] // 2
            a = (F.silu(gu[:, :Fh].float()) * gu[:, Fh:].float()).to(x.dtype)
            delta = _lin(a, lw.down)
        h = (h.float() + delta.float()).to(h.dtype)
    x = _rms(h, model.final_norm, cfg.rms_norm_eps)
    return _lin(x, model.lm_head).float()[:, :cfg.vocab_size]


def greedy_generate(model: TransformerLM, prompt: list[int], n: int) -> list[int]:
    toks = list(prompt)
    out = []
    for _ in range(n):
        nxt = int(dense_logits(model, toks)[-1].argmax())
        out.append(nxt)
        toks.append(nxt)
    return out
