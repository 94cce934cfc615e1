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

import os

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.parallel import state as pstate

# Steps of up to this many tokens run the expert MLP on the grouped weight-streaming kernel. Unlike the dense
# projections it is not limited to 128 rows: each expert's segment is cut into 64-row tiles, so an expert's weights
# are streamed once per 64 of ITS rows (top-2 of 8 at T = 256 is ~64 rows per expert). Measured
# (profiles/r02/moe_stream_max_t_ab.jsonl, moe_bench_stream512.log): T = 512 layer 1,252 vs 1,391 us on the LDS-tiled
# grouped GEMM; Mixtral-8x7B 128-thread bench 4,783 (128) -> 4,958 tok/s (640 = 128 decodes + the TPOT guard's 512
# prefill tokens), TTFT 62 -> 58 ms. Env KAFKA_MOE_STREAM_MAX_T overrides.
MOE_STREAM_MAX_T = int(os.environ.get("KAFKA_MOE_STREAM_MAX_T", "640"))


def route(logits: torch.Tensor, k: int):
    """softmax -> top-k -> renormalise (Mixtral). Returns (weights f32 [T,k], experts int64 [T,k])."""
    p = torch.softmax(logits.float(), dim=-1)
    w, e = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, e


class MoEBlock:
    def __init__(self, model):
        self.model = model
        # expert all-to-all dispatch/combine instead of the all-reduce combine (opt-in, see _a2a)
        self.dp = model.dp_attention  # tokens are this rank's own (not replicated): dispatch all, no all-gather
        self.a2a = self.dp or os.environ.get("KAFKA_MOE_A2A", "0") == "1"
        cfg = model.cfg
        self.E = cfg.num_experts
        self.k = cfg.num_experts_per_tok
        self.F = cfg.intermediate_size
        self.ep = model.ep
        self.r = model.ep_rank
        self.e_local = self.E // self.ep
        self.e0 = self.r * self.e_local

    def __call__(self, x: torch.Tensor, lw) -> torch.Tensor:
        T, d = x.shape
        logits = F.linear(x, lw.router)
        r = ops.moe_route(logits, self.k)
        if self.ep > 1 and self.a2a:
            return self._a2a(x, lw, r)
        if self.model.stream and lw.w13_t is not None and T <= MOE_STREAM_MAX_T:
            # decode-sized steps: expert weights streamed from their wave-tiled copies, SwiGLU fused into the gate_up
            # epilogue, weighted combine fused into the down epilogue (csrc/wstream_gemm.hip, grouped variant)
            a = ops.grouped_stream_glu(x, lw.w13_t, r, e_lo=self.e0)
            out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
            ops.grouped_stream_combine(a, lw.w2_t, r, T, out, e_lo=self.e0)
            return self._finish(out, x.dtype)
        # gate_up for every (token, expert) entry routed to a local expert, rows gathered from x by the kernel
        h = ops.grouped_gemm(x, lw.w13, r, gather=True, e_lo=self.e0)
        a = ops.silu_mul(h)
        # down projection with the routing-weighted scatter-combine fused into the epilogue
        out = torch.zeros(T, d, dtype=torch.float32, device=x.device)
        ops.grouped_gemm(a, lw.w2, r, gather=False, e_lo=self.e0, combine_out=out)
        return self._finish(out, x.dtype)

    def _finish(self, out: torch.Tensor, dtype) -> torch.Tensor:
        """The fp32 combine buffer [T, d] as the layer's delta, handed on as a one-split slab [1, T, d] (the next add +
        RMSNorm sums slabs while loading — no separate fp32 -> bf16 pass). Expert-parallel ranks hold partial sums
        over their own experts: the decoder's layer seam all-reduces them (``reduced`` is False)."""
        return out.unsqueeze(0)

    @property
    def reduced(self) -> bool:
        """True if the layer output is already complete on every rank (the all-to-all path combines in place)."""
        return self.ep == 1 or bool(self.a2a)


    # ------------------------------------------------------------------------------------------------------------
    def _a2a(self, x: torch.Tensor, lw, r) -> torch.Tensor:
        """Expert parallelism with an all-to-all dispatch and combine (``KAFKA_MOE_A2A=1``; BASELINE config 5's
        "expert all-to-all"), device-side end to end: no host synchronisation, capturable into a hipGraph.

        Every rank holds all T tokens (replicated after the attention all-reduce) and computes the same routing.
        Rank q OWNS tokens [q Tl, (q+1) Tl). ``ops.ep_dispatch`` (csrc/moe.hip) packs each owned (token, expert)
        pair into the block of the rank that holds the expert — fixed capacity C = Tl min(k, El) slots per
        destination plus metadata rows carrying the count and each slot's local expert — so the transport needs no
        split sizes from the host. Transport: the custom IPC all-to-all (parallel/custom_allreduce.py, the same
        buffers and epochs as the decode all-reduce) when the image fits its buffer, else ``all_to_all_single``
        (RCCL; gloo when the ranks share one GPU). The expert ranks route the received slots on the device
        (``ops.ep_recv_route``), run their local experts with the same grouped kernels as the all-reduce path
        (weights 1), send the rows back, the owners apply the routing weights (``ops.ep_combine``) and the owned
        rows are all-gathered into the replicated [T, d] the next layer expects. With tensor-parallel attention
        this moves more bytes than the default all-reduce combine (capacity padding + the all-gather), so it is
        opt-in; it is the dispatch/combine a data-parallel attention layout needs, where tokens are not
        replicated."""
        from kafka_llm_service_amd.parallel import comm

        T, d = x.shape
        ep, q, k, El = self.ep, self.r, self.k, self.e_local
        st = pstate.get()
        grp = st.ep_group if self.dp else st.tp_group
        if self.dp:  # DP attention: all T tokens are this rank's; capacity from the group's largest step
            Tl, C, MR = ops.ep_layout(max(T, self.model.ep_t_cap) * ep, ep, k, El, d)
            lo, n_own = 0, T
        else:
            Tl, C, MR = ops.ep_layout(T, ep, k, El, d)
            lo, hi = min(T, q * Tl), min(T, (q + 1) * Tl)
            n_own = hi - lo
        img, slot = ops.ep_dispatch(x, r.topk_e, lo, n_own, El, ep, C, MR)
        car = comm.get_custom(grp)
        if car is not None and not car.fits_bytes(img.numel() * img.element_size()):
            car = None

        def exchange(send: torch.Tensor) -> torch.Tensor:
            recv = torch.empty_like(send)
            if car is not None:
                return car.all_to_all(send, recv)
            return comm.all_to_all_single(recv, send, grp)

        recv = exchange(img)
        rr = ops.ep_recv_route(recv, C, El)
        rows = recv.view(-1, d)
        y = torch.zeros(rows.shape[0], d, dtype=torch.float32, device=x.device)
        if self.model.stream and lw.w13_t is not None and rows.shape[0] <= MOE_STREAM_MAX_T:
            a = ops.grouped_stream_glu(rows, lw.w13_t, rr, e_lo=0)
            ops.grouped_stream_combine(a, lw.w2_t, rr, rows.shape[0], y, e_lo=0)
        else:
            h = ops.grouped_gemm(rows, lw.w13, rr, gather=True, e_lo=0)
            ops.grouped_gemm(ops.silu_mul(h), lw.w2, rr, gather=False, e_lo=0, combine_out=y)
        back = exchange(y.to(x.dtype).view(ep, C + MR, d))
        if self.dp:
            out = torch.empty(T, d, dtype=x.dtype, device=x.device)
            return ops.ep_combine(back, slot, r.topk_w, 0, T, out)
        own = torch.empty(Tl, d, dtype=x.dtype, device=x.device)
        if n_own < Tl:
            own[n_own:].zero_()  # past the last token (sliced off below; kept finite)
        ops.ep_combine(back, slot, r.topk_w, lo, n_own, own)
        full = torch.empty(ep * Tl, d, dtype=x.dtype, device=x.device)
        if car is not None and car.fits_bytes(own.numel() * own.element_size()):
            car.all_gather(own, full)
        else:
            comm.all_gather_into(full, own, ep, grp)
        return full[:T]

    def serve_idle(self, lw, d: int, dtype, device) -> None:
        """DP attention, a rank with no tokens this step: its experts still serve the other ranks' tokens — the
        same collectives as _a2a with an empty dispatch (every destination block has count 0)."""
        from kafka_llm_service_amd.parallel import comm

        ep, k, El = self.ep, self.k, self.e_local
        grp = pstate.get().ep_group
        Tl, C, MR = ops.ep_layout(self.model.ep_t_cap * ep, ep, k, El, d)
        x = torch.zeros(1, d, dtype=dtype, device=device)
        te = torch.zeros(1, k, dtype=torch.int32, device=device)
        img, _ = ops.ep_dispatch(x, te, 0, 0, El, ep, C, MR)
        car = comm.get_custom(grp)
        if car is not None and not car.fits_bytes(img.numel() * img.element_size()):
            car = None

        def exchange(send):
            recv = torch.empty_like(send)
            return car.all_to_all(send, recv) if car is not None else comm.all_to_all_single(recv, send, grp)

        recv = exchange(img)
        rr = ops.ep_recv_route(recv, C, El)
        rows = recv.view(-1, d)
        y = torch.zeros(rows.shape[0], d, dtype=torch.float32, device=device)
        if self.model.stream and lw.w13_t is not None and rows.shape[0] <= MOE_STREAM_MAX_T:
            a = ops.grouped_stream_glu(rows, lw.w13_t, rr, e_lo=0)
            ops.grouped_stream_combine(a, lw.w2_t, rr, rows.shape[0], y, e_lo=0)
        else:
            h = ops.grouped_gemm(rows, lw.w13, rr, gather=True, e_lo=0)
            ops.grouped_gemm(ops.silu_mul(h), lw.w2, rr, gather=False, e_lo=0, combine_out=y)
        exchange(y.to(dtype).view(ep, C + MR, d))
