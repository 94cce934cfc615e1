"""Mixtral sparse-MoE block: top-2 router, expert-sorted dispatch, grouped expert GEMMs, weighted combine.

Expert parallelism runs over the TP group: rank r owns experts [r E/ep, (r+1) E/ep). Attention is tensor-parallel,
so every rank of the group already holds all T token activations after the O-projection all-reduce; each rank runs
its own experts over the tokens routed to them and the per-rank partial outputs are summed by the same all-reduce
that a dense row-parallel MLP would use (one collective per layer, [T, d] bf16). With ep = 1 the whole block is
local (Mixtral 8x7B bf16 = 93 GB fits one 288 GB MI355X).

Per layer: router GEMM (hipBLASLt) -> ``ops.moe_route`` (HIP, one workgroup: softmax + top-k + renormalise + stable
expert sort, no host sync) -> ``ops.grouped_gemm`` gate_up (HIP MFMA, A rows gathered through the permutation) ->
``ops.silu_mul`` -> ``ops.grouped_gemm`` down with the routing-weighted scatter-combine fused into its epilogue
(fp32 atomics onto a zeroed [T, d] buffer). On CPU the same calls run the fp32 references of ``ops/reference.py``.
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
        self.model = model
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
        r = ops.moe_route(logits, self.k)
        if self.model.stream and lw.w13_t is not None and T <= ops.STREAM_MAX_M:
            # decode-sized steps: expert weights streamed from their wave-tiled copies, SwiGLU fused into the gate_up
            # epilogue, weighted combine fused into the down epilogue (csrc/wstream_gemm.hip, grouped variant)
            a = ops.grouped_stream_glu(x, lw.w13_t, r, e_lo=self.e0)
            out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
            ops.grouped_stream_combine(a, lw.w2_t, r, T, out, e_lo=self.e0)
            out = out.to(x.dtype)
            return pstate.tp_all_reduce(out) if self.ep > 1 else out
        # gate_up for every (token, expert) entry routed to a local expert, rows gathered from x by the kernel
        h = ops.grouped_gemm(x, lw.w13, r, gather=True, e_lo=self.e0)
        a = ops.silu_mul(h)
        # down projection with the routing-weighted scatter-combine fused into the epilogue
        out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
        ops.grouped_gemm(a, lw.w2, r, gather=False, e_lo=self.e0, combine_out=out)
        out = out.to(x.dtype)
        if self.ep > 1:
            out = pstate.tp_all_reduce(out)
        return out
