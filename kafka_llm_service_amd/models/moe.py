"""Mixtral sparse-MoE block: top-2 router, expert-sorted dispatch, grouped expert GEMMs, weighted combine.

Expert parallelism runs over the TP group: rank r owns experts [r E/ep, (r+1) E/ep). Attention is tensor-parallel,
so every rank of the group already holds all T token activations after the O-projection all-reduce; each rank runs
its own experts over the tokens routed to them and the per-rank partial outputs are summed by the same all-reduce
that a dense row-parallel MLP would use (one collective per layer, [T, d] bf16). With ep = 1 the whole block is
local (Mixtral 8x7B bf16 = 93 GB fits one 288 GB MI355X).

GPU path: ``ops.moe_route`` (HIP: softmax + top-k + renormalise + expert histogram + permutation, one kernel) and
``ops.grouped_gemm`` (HIP MFMA grouped GEMM over the expert-sorted rows) when the extension provides them; the CPU
path is the plain PyTorch reference of the same math.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.parallel import state as pstate


def route(logits: torch.Tensor, k: int):
    """softmax -> top-k -> renormalise (Mixtral). Returns (weights f32 [T,k], experts int64 [T,k])."""
    p = torch.softmax(logits.float(), dim=-1)
    w, e = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, e


class MoEBlock:
    def __init__(self, model):
        cfg = model.cfg
        self.E = cfg.num_experts
        self.k = cfg.num_experts_per_tok
        self.F = cfg.intermediate_size
        self.ep = model.tp
        self.r = model.tp_rank
        self.e_local = self.E // self.ep
        self.e0 = self.r * self.e_local

    def __call__(self, x: torch.Tensor, lw) -> torch.Tensor:
        T, d = x.shape
        logits = F.linear(x, lw.router)
        w, e = route(logits, self.k)
        out = self._experts(x, w, e, lw)
        if self.ep > 1:
            out = pstate.tp_all_reduce(out)
        return out

    def _experts(self, x, w, e, lw) -> torch.Tensor:
        T, d = x.shape
        flat_e = e.reshape(-1)
        flat_w = w.reshape(-1)
        tok = torch.arange(T, device=x.device).repeat_interleave(self.k)
        local = (flat_e >= self.e0) & (flat_e < self.e0 + self.e_local)
        le = flat_e[local] - self.e0
        order = torch.argsort(le, stable=True)
        le, ltok, lw_ = le[order], tok[local][order], flat_w[local][order]
        counts = torch.bincount(le, minlength=self.e_local)
        xs = x.index_select(0, ltok)
        if x.is_cuda and hasattr(ops, "grouped_gemm") and ops.has_grouped_gemm():
            offs = torch.zeros(self.e_local + 1, dtype=torch.int32, device=x.device)
            offs[1:] = torch.cumsum(counts, 0)
            h = ops.grouped_gemm(xs, lw.w13, offs)
            a = ops.silu_mul(h)
            y = ops.grouped_gemm(a, lw.w2, offs)
        else:
            y = torch.empty(xs.shape[0], d, dtype=x.dtype, device=x.device)
            start = 0
            for j, c in enumerate(counts.tolist()):
                if c:
                    h = F.linear(xs[start:start + c], lw.w13[j])
                    y[start:start + c] = F.linear(ops.silu_mul(h), lw.w2[j])
                start += c
        out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
        out.index_add_(0, ltok, y.float() * lw_[:, None])
        return out.to(x.dtype)
