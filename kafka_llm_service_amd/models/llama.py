"""Llama-3 / Llama-3.1 / Mixtral decoder for the serving engine (TP-sharded, paged KV, CDNA4 kernels).

Per layer (SURVEY.md §3.2 "Target equivalent"):
    fused_add_rmsnorm -> QKV GEMM (column-parallel) -> rope_kv_write (RoPE + paged KV write, HIP)
    -> paged attention (decode / cascade / chunked prefill, HIP MFMA) -> O GEMM (row-parallel) -> [TP all-reduce]
    -> fused_add_rmsnorm -> gate_up GEMM (column-parallel) -> silu_mul (HIP) -> down GEMM (row-parallel)
    -> [TP all-reduce]                                     (Mixtral: router -> expert MLPs, models/moe.py)
Decode-sized steps (T <= 128) run every projection on the weight-streaming MFMA kernel (``ops/csrc/wstream_gemm.hip``,
wave-tiled weight copies, SwiGLU fused into gate_up; the grouped variant for Mixtral's experts); 129..256-row mixed
steps run qkv / o / down on the skinny MFMA GEMM (``ops/csrc/skinny_gemm.hip``, SKINNY below); other prefill-sized
steps use hipBLASLt through ``torch.nn.functional.linear`` (bf16, fp32 accumulate). Norm / RoPE / attention / sampling run
in the hand-written kernels of ``ops/csrc``.

Weights are stored HF-style ``[out, in]`` so safetensors checkpoints load without transposes; random init (seeded,
synthetic benchmarks — no checkpoints are downloadable here) is the default.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.models.attention import AttnMeta, paged_attention
from kafka_llm_service_amd.models.config import ModelConfig
from kafka_llm_service_amd.parallel import state as pstate

# TP decode seam overlap (KAFKA_TP_OVERLAP=1): the row-parallel O / down projection of a decode-sized step is
# computed in two column halves; half 0's all-reduce runs on a second HIP stream (into a persistent buffer) while half
# 1's GEMM streams its weights on the main one, then ONE launch on the main stream all-reduces half 1, joins half 0
# (read in place: no concatenation), adds the residual and applies the next RMSNorm (csrc/allreduce.hip, the fused
# kernel's ``pre`` columns). Unlike a split of the batch into two micro-batches it reads every weight once (decode
# GEMMs are weight-bound), and the per-element sums are those of the one-shot all-reduce. Captured hipGraphs record
# the fork/join. Off by default: the gain needs TP over xGMI to measure (ranks sharing one GPU overlap nothing).
TP_OVERLAP = os.environ.get("KAFKA_TP_OVERLAP", "0") == "1"

# Projections of 129..256-row steps (decode + a new turn's prefill) that run on the skinny MFMA GEMM
# (ops.linear_skinny, csrc/skinny_gemm.hip) instead of hipBLASLt: env KAFKA_SKINNY, a comma list of qkv / o / down
# ("" = none; "+" also separates). gate_up stays on hipBLASLt (faster there). Same-box A/B, 2 interleaved rounds:
# 7,857 (none) -> 7,924 tok/s (o+down or all three), profiles/r03/skinny_gemm/bench_ab_wired.jsonl.
# Prefill-sized TP seams whose message exceeds the custom all-reduce's buffer (RCCL): the row-parallel GEMM and the
# all-reduce are pipelined over row blocks of at least PIPE_ROWS tokens, at most PIPE_CHUNKS blocks
# (comm.pipelined_linear_all_reduce; env KAFKA_TP_PIPE_CHUNKS, 1 = off). At Llama-3-70B TP = 8 a 2k-token chunk has
# 160 such seams of 32 MiB each; with the pipeline only the last block's all-reduce is left exposed.
PIPE_CHUNKS = max(1, int(os.environ.get("KAFKA_TP_PIPE_CHUNKS", "4")))
PIPE_ROWS = 256
SKINNY = frozenset(p for p in os.environ.get("KAFKA_SKINNY", "qkv,o,down").replace("+", ",").split(",")
                   if p in ("qkv", "o", "down", "gate_up"))  # gate_up: fused SwiGLU epilogue (A/B, not default)
# Fused decode layer (forward -> _forward_fused; env KAFKA_FUSED_DECODE=1): 6 launches per layer instead of 9 —
# deferred RMSNorm and RoPE + KV write inside the streaming GEMMs' split-K finishers. Correct (fp32-reference and
# buffer-reuse tests) but OFF by default: each finisher is one workgroup reducing its column block's slabs at the
# launch's tail (~220 KB through one CU at ~64 B/clk, plus drain / ticket / load round trips: 4-7 us), which costs
# more than the RMSNorm / RoPE launches it removes — headline 8,231 vs 8,671 tok/s same box
# (profiles/r06/fused/README.md).
FUSED = os.environ.get("KAFKA_FUSED_DECODE", "0") == "1"
_OVL: dict = {}
_SEAM_DONE = object()  # forward(): the previous layer's overlapped seam already produced this layer's input


def _overlap_stream(dev: torch.device):
    s = _OVL.get(dev)
    if s is None:
        s = _OVL[dev] = (torch.cuda.Stream(device=dev), [torch.cuda.Event() for _ in range(3)])
    return s


@dataclass
class StepInput:
    """Device tensors of one engine step."""
    tokens: torch.Tensor          # int64 [T]
    positions: torch.Tensor       # int64 [T]
    slot_mapping: torch.Tensor    # int64 [T] (-1 = do not write KV)
    attn: AttnMeta
    logit_rows: torch.Tensor      # int64 [n] rows whose next-token logits are needed


class LayerWeights:
    __slots__ = ("input_norm", "post_norm", "qkv", "o", "gate_up", "down", "router", "w13", "w2", "expert_ids",
                 "qkv_t", "o_t", "gate_up_t", "down_t", "glu", "w13_t", "w2_t")
    STREAMED = ("qkv", "o", "gate_up", "down")  # projections with a wave-tiled copy for the decode GEMM

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)


class TransformerLM:
    """Functional model: holds weight tensors + the RoPE table and runs one step over paged KV caches."""

    def __init__(self, cfg: ModelConfig, device: torch.device, dtype=torch.bfloat16, tp: int = 1, tp_rank: int = 0,
                 max_positions: int | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp, self.tp_rank = tp, tp_rank
        # expert parallelism: over the TP group by default; DP attention (enable_dp_attention) keeps attention
        # unsharded (tp = 1, every rank its own sequences) and shards the experts over a separate group
        self.ep, self.ep_rank = tp, tp_rank
        self.dp_attention = False
        self.ep_t_cap = 0  # DP attention: max tokens of this step over the group (the all-to-all capacity)
        if cfg.num_heads % tp or cfg.num_kv_heads % tp:
            raise ValueError(f"heads ({cfg.num_heads}/{cfg.num_kv_heads}) not divisible by tp={tp}")
        self.hq = cfg.num_heads // tp
        self.hkv = cfg.num_kv_heads // tp
        self.D = cfg.head_dim
        self.ffn = cfg.intermediate_size // tp if not cfg.num_experts else cfg.intermediate_size
        self.vocab_local = (cfg.vocab_size + tp - 1) // tp
        self.layers: list[LayerWeights] = [LayerWeights() for _ in range(cfg.num_layers)]
        self.embed = None       # [V_local, d]
        self.lm_head = None     # [V_local, d]
        self.final_norm = None  # [d]
        maxp = max_positions or cfg.max_position_embeddings
        self.cos_sin = ops.rope_cos_sin(maxp, self.D, cfg.rope_theta, cfg.rope_scaling, device=self.device)
        self.scale = self.D ** -0.5
        self.moe = None
        self.lm_head_t = None
        self.stream = False  # decode GEMMs on the weight-streaming kernel (enable_stream_weights)
        self.tiled_only = False  # row-major dense weights dropped (enable_stream_weights(tiled_only=True))
        self.stream_max_m = ops.STREAM_MAX_M  # rows up to which a step's projections stream
        self._fused_shapes = None  # whether the fused decode layer applies to this model (decided on first use)

    def enable_dp_attention(self, ep: int, ep_rank: int) -> None:
        """Data-parallel attention for a MoE model (call before the weights are created): attention, norms and the
        vocabulary stay whole on every rank (tp must be 1), each rank runs its own sequences, and the experts are
        sharded over the ``ep`` ranks of ``parallel.state``'s EP group with the device-side all-to-all dispatch and
        combine (models/moe.py) — the layout where expert all-to-all beats an all-reduce combine: every rank sends
        only its own tokens' rows, and attention/KV are split instead of replicated."""
        if self.tp != 1 or not self.cfg.num_experts or self.cfg.num_experts % ep:
            raise ValueError("DP attention needs tp = 1 and experts divisible by the EP size")
        self.ep, self.ep_rank, self.dp_attention = ep, ep_rank, True

    def dp_idle_step(self) -> None:
        """DP attention: a group step in which this rank has no tokens — only its experts' share of every MoE
        layer's all-to-all runs (the other ranks' tokens routed here), in layer order like a real forward."""
        for lw in self.layers:
            self.moe.serve_idle(lw, self.cfg.hidden_size, self.dtype, self.device)

    # ------------------------------------------------------------------------------------------------------------
    def stream_weight_bytes(self) -> int:
        """Bytes enable_stream_weights would add (the wave-tiled copies; 0 in tiled-only mode)."""
        n = 0
        for lw in self.layers:
            for name in LayerWeights.STREAMED:
                w = getattr(lw, name)
                if w is not None and ops.stream_plan(1, w.shape[0], w.shape[1]) is not None:
                    n += w.numel() * w.element_size()
            for name in ("w13", "w2"):
                w = getattr(lw, name)
                if w is not None and ops.stream_moe_supported(w.shape[1], w.shape[2]):
                    n += w.numel() * w.element_size()
        if self.lm_head is not None and ops.stream_plan(1, self.lm_head.shape[0], self.lm_head.shape[1]) is not None:
            n += self.lm_head.numel() * self.lm_head.element_size()
        return n

    def enable_stream_weights(self, tiled_only: bool = False) -> int:
        """Keep a wave-tiled copy of every dense projection and of the lm_head (ops.tile_weight) so decode-sized
        steps (T <= ops.STREAM_MAX_M) run the weight-streaming MFMA GEMM (csrc/wstream_gemm.hip) instead of
        hipBLASLt; prefill-sized steps keep the row-major weights. Costs one more copy of those weights (16 GB for
        Llama-3-8B: the HBM of an MI355X has room, and the KV pool is sized after this). Returns the added bytes.

        ``tiled_only``: when the second copy does not fit (Llama-3-70B on one GPU), the row-major dense projections
        and the lm_head are dropped after tiling (no extra memory) and prefill-sized steps untile one weight at a
        time into a transient buffer for hipBLASLt (``_dense``); MoE experts keep their row-major layout only
        (grouped GEMM at every step size — a tiled expert copy would be the 90 GB second copy this mode avoids)."""
        added = 0
        for lw in self.layers:
            for name in LayerWeights.STREAMED:
                w = getattr(lw, name)
                if w is not None and ops.stream_plan(1, w.shape[0], w.shape[1]) is not None:
                    glu = name == "gate_up" and w.shape[0] % 64 == 0
                    setattr(lw, name + "_t", ops.tile_weight(w, glu=glu))
                    if name == "gate_up":
                        lw.glu = glu
                    if tiled_only:
                        setattr(lw, name, None)
                        del w
                    else:
                        added += w.numel() * w.element_size()
            if not tiled_only and lw.w13 is not None and \
                    ops.stream_moe_supported(lw.w13.shape[1], lw.w13.shape[2]) and \
                    ops.stream_moe_supported(lw.w2.shape[1], lw.w2.shape[2]):
                lw.w13_t = ops.tile_experts(lw.w13, glu=True)  # expert MLPs: grouped streaming kernel
                lw.w2_t = ops.tile_experts(lw.w2)
                added += (lw.w13.numel() + lw.w2.numel()) * lw.w13.element_size()
        if ops.stream_plan(1, self.lm_head.shape[0], self.lm_head.shape[1]) is not None:
            self.lm_head_t = ops.tile_weight(self.lm_head)
            if tiled_only:
                self.lm_head = None
            else:
                added += self.lm_head_t.numel() * self.lm_head_t.element_size()
        self.stream = True
        self.tiled_only = tiled_only
        # tiled-only: any larger step would untile every projection for hipBLASLt, so the streaming kernel takes
        # steps up to its 256-row limit (two row tiles beyond 128) — slower than hipBLASLt there, far cheaper than
        # untiling
        self.stream_max_m = ops.STREAM_KERNEL_MAX_M if tiled_only else ops.STREAM_MAX_M
        if tiled_only and self.device.type == "cuda":
            torch.cuda.empty_cache()
        return added

    def _linear(self, x: torch.Tensor, w: torch.Tensor, wt: torch.Tensor | None, max_splits: int = 8,
                kind: str = ""):
        """x @ w^T: the weight-streaming kernel for decode-sized x (bf16 or a split-K slab out), the skinny MFMA GEMM
        for 129..256 rows of the projections in SKINNY, else hipBLASLt."""
        M = x.shape[0]
        if self.stream and wt is not None:
            if 0 < M <= self.stream_max_m:
                return ops.linear_stream(x, wt, max_splits)
            if kind in SKINNY and ops.skinny_plan(M, wt.shape[0] * 32, x.shape[1], max_splits):
                return ops.linear_skinny(x, wt, max_splits)
        return F.linear(x, self._dense(w, wt))

    @staticmethod
    def _dense(w: torch.Tensor | None, wt: torch.Tensor | None, glu: bool = False) -> torch.Tensor:
        """The row-major weight for hipBLASLt: the stored one, or (tiled-only mode) a transient untiled copy."""
        return w if w is not None else ops.untile_weight(wt, glu=glu)

    def forward(self, inp: StepInput, k_caches: list[torch.Tensor], v_caches: list[torch.Tensor],
                gather: bool = True) -> torch.Tensor:
        """Returns logits [n, V] (bf16) for ``inp.logit_rows`` — with ``gather=False`` this rank's vocab shard
        [n, V_local] instead (the caller all-gathers: a captured decode graph ends before that collective).

        On decode-sized steps the projections return split-K slabs (fp32 [S, T, n], see ops.linear_stream) which
        rope_kv_write / silu_mul / fused_add_rmsnorm consume directly. Under TP every layer seam (O projection, MLP
        down projection) is ONE call: all-reduce of the row-parallel partial sums + residual add + the next RMSNorm
        (the custom xGMI all-reduce fuses all three when the message fits its buffer, parallel/comm.py)."""
        cfg = self.cfg
        T = inp.tokens.shape[0]
        if self._fused_ok(T, k_caches):
            return self._forward_fused(inp, k_caches, v_caches, gather)
        h = self._embed(inp.tokens)
        residual = h
        x = torch.empty_like(h)
        q = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
        attn_out = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
        eps = cfg.rms_norm_eps
        tp = self.tp > 1
        delta, pending = None, False
        for i, lw in enumerate(self.layers):
            if delta is _SEAM_DONE:
                pass  # the previous layer's overlapped down seam already wrote residual and x
            elif delta is None:
                ops.rmsnorm(h, lw.input_norm, eps, out=x)
                # the embedding is a fresh tensor at TP = 1 (the residual stream can own it); under TP it may be the
                # all-reduce's persistent buffer
                residual = h if self.tp == 1 else h.clone()
            elif pending:
                pstate.tp_all_reduce_add_rmsnorm(delta, residual, lw.input_norm, eps, out=x)
            else:
                ops.fused_add_rmsnorm(delta, residual, lw.input_norm, eps, out=x)
            qkv = self._linear(x, lw.qkv, lw.qkv_t, kind="qkv")
            ops.rope_kv_write(qkv, inp.positions, self.cos_sin, q, k_caches[i], v_caches[i], inp.slot_mapping,
                              self.hq, self.hkv)
            paged_attention(q, k_caches[i], v_caches[i], inp.attn, attn_out)
            if tp and self._can_overlap(T, lw.o_t):
                self._overlapped_seam(attn_out.view(T, -1), lw.o_t, residual, lw.post_norm, eps, x)
            elif tp and self._can_pipe(T, lw.o, lw.o_t):
                o = pstate.tp_linear_all_reduce(attn_out.view(T, -1), self._dense(lw.o, lw.o_t), self._pipe_chunks(T))
                ops.fused_add_rmsnorm(o, residual, lw.post_norm, eps, out=x)
            else:
                o = self._linear(attn_out.view(T, -1), lw.o, lw.o_t, kind="o")
                if tp:
                    pstate.tp_all_reduce_add_rmsnorm(o, residual, lw.post_norm, eps, out=x)
                else:
                    ops.fused_add_rmsnorm(o, residual, lw.post_norm, eps, out=x)
            if lw.router is not None:
                delta = self.moe(x, lw)
                pending = tp and not self.moe.reduced
                continue
            if self.stream and lw.glu and 0 < T <= self.stream_max_m:
                a = ops.linear_glu(x, lw.gate_up_t)  # SwiGLU in the GEMM epilogue (or on its slabs)
            elif (self.stream and lw.glu and "gate_up" in SKINNY and lw.gate_up_t is not None
                  and ops.skinny_plan(T, lw.gate_up_t.shape[0] * 32, x.shape[1])):
                a = ops.linear_skinny(x, lw.gate_up_t, glu=True)  # fused SwiGLU (one split) or gate | up slabs
                if ops.is_slab(a):
                    a = ops.silu_mul(a)
            else:
                a = ops.silu_mul(F.linear(x, self._dense(lw.gate_up, lw.gate_up_t, bool(lw.glu))))
            if tp and self._can_overlap(T, lw.down_t) and i + 1 < len(self.layers):
                # the next layer's input RMSNorm is the seam's normalisation: delta is consumed here
                self._overlapped_seam(a, lw.down_t, residual, self.layers[i + 1].input_norm, eps, x)
                delta, pending = _SEAM_DONE, False
            elif tp and self._can_pipe(T, lw.down, lw.down_t):
                delta = pstate.tp_linear_all_reduce(a, self._dense(lw.down, lw.down_t), self._pipe_chunks(T))
                pending = False  # already reduced: the next seam is a plain add + RMSNorm
            else:
                delta = self._linear(a, lw.down, lw.down_t, kind="down")
                pending = tp
        if pending:
            delta = pstate.tp_all_reduce(delta)
        rows = inp.logit_rows
        d_sel = delta.index_select(1 if ops.is_slab(delta) else 0, rows)
        r_sel = residual.index_select(0, rows)
        hf = ops.fused_add_rmsnorm(d_sel, r_sel, self.final_norm, eps)
        logits = self._linear(hf, self.lm_head, self.lm_head_t, max_splits=1)
        if not gather:
            return logits
        if tp:
            logits = pstate.tp_all_gather_lastdim(logits)
        return logits[:, :cfg.vocab_size]

    def _fused_ok(self, T: int, k_caches: list[torch.Tensor]) -> bool:
        """Decode-sized TP = 1 dense steps run the fused layer (FUSED above) when every projection has its wave-tiled
        copy, the KV cache is bf16 with 128-dim heads and the shapes fit the fused epilogues."""
        if not (FUSED and self.stream and self.tp == 1 and not self.dp_attention and 0 < T <= self.stream_max_m):
            return False
        if self._fused_shapes is None:
            lw0 = self.layers[0]
            ok = all(lw.router is None and lw.glu and lw.qkv_t is not None and lw.o_t is not None and
                     lw.down_t is not None for lw in self.layers)
            self._fused_shapes = ok and self.D == 128 and not ops.is_fp8_cache(k_caches[0]) and \
                ops.stream_plan(1, self.cfg.hidden_size, lw0.down_t.shape[1] * 16) is not None
        if not self._fused_shapes:
            return False
        lw0 = self.layers[0]
        return ops.fin_supported(T, self.cfg.hidden_size, lw0.qkv_t.shape[0] * 32, lw0.gate_up_t.shape[0] * 32, self.D) \
            and ops.stream_plan(T, self.cfg.hidden_size, lw0.down_t.shape[1] * 16) is not None

    def _forward_fused(self, inp: StepInput, k_caches: list[torch.Tensor], v_caches: list[torch.Tensor],
                       gather: bool) -> torch.Tensor:
        """The decode layer as 6 launches (qkv + RoPE/KV write -> cascade -> decode -> o + residual add -> gate_up +
        SwiGLU -> down + residual add): RMSNorm is deferred into the consuming GEMMs (the residual producer writes
        bf16(h * w) and per-column-block sums of h^2, the consumer scales rows by rsqrt(mean h^2 + eps)) and RoPE +
        the paged KV write run in the QKV GEMM's split-K finisher (ops.linear_res / linear_qkv_rope / linear_glu_rs,
        csrc/wstream_gemm.hip FIN_*). Only layer 0's input norm (from the embedding) and the final norm stay kernels."""
        cfg = self.cfg
        T = inp.tokens.shape[0]
        d, eps = cfg.hidden_size, cfg.rms_norm_eps
        residual = self._embed(inp.tokens)  # a fresh tensor at TP = 1: the residual stream owns it
        x = torch.empty_like(residual)
        q = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
        attn_out = torch.empty(T, self.hq, self.D, dtype=self.dtype, device=self.device)
        ss = torch.empty(2, d // 128, T, dtype=torch.float32, device=self.device)
        ops.rmsnorm(residual, self.layers[0].input_norm, eps, out=x)
        ss_in, delta = None, None
        L = len(self.layers)
        for i, lw in enumerate(self.layers):
            ops.linear_qkv_rope(x, lw.qkv_t, ss_in, eps, inp.positions, self.cos_sin, q, k_caches[i], v_caches[i],
                                inp.slot_mapping, self.hq, self.hkv)
            paged_attention(q, k_caches[i], v_caches[i], inp.attn, attn_out)
            ops.linear_res(attn_out.view(T, -1), lw.o_t, residual, lw.post_norm, x, ss[0], pool="fin_o")
            a = ops.linear_glu_rs(x, lw.gate_up_t, ss[0], eps)
            if i + 1 < L:
                ops.linear_res(a, lw.down_t, residual, self.layers[i + 1].input_norm, x, ss[1], pool="fin_down")
                ss_in = ss[1]
            else:
                delta = self._linear(a, lw.down, lw.down_t, kind="down")
        rows = inp.logit_rows
        d_sel = delta.index_select(1 if ops.is_slab(delta) else 0, rows)
        hf = ops.fused_add_rmsnorm(d_sel, residual.index_select(0, rows), self.final_norm, eps)
        logits = self._linear(hf, self.lm_head, self.lm_head_t, max_splits=1)
        return logits if not gather else logits[:, :cfg.vocab_size]

    def _can_pipe(self, T: int, w: torch.Tensor | None, wt: torch.Tensor | None) -> bool:
        """A prefill-sized seam that goes to the library all-reduce (beyond the custom all-reduce's buffer) and is
        long enough to pipeline its GEMM against it."""
        if PIPE_CHUNKS < 2 or T < 2 * PIPE_ROWS or (self.stream and T <= self.stream_max_m):
            return False
        car = pstate.custom_ar()
        n = (w.shape[0] if w is not None else wt.shape[0] * 32)
        return car is None or T * n * 2 > car.max_bytes

    def _pipe_chunks(self, T: int) -> int:
        return max(2, min(PIPE_CHUNKS, T // PIPE_ROWS))

    def _can_overlap(self, T: int, wt: torch.Tensor | None) -> bool:
        if not (TP_OVERLAP and self.stream and wt is not None and 0 < T <= self.stream_max_m and self.device.type == "cuda"):
            return False
        car = pstate.custom_ar()
        return car is not None and wt.shape[0] % 2 == 0 and T * wt.shape[0] * 32 * 2 <= car.max_bytes

    def _overlapped_seam(self, a: torch.Tensor, wt: torch.Tensor, residual: torch.Tensor, norm_w: torch.Tensor,
                         eps: float, out: torch.Tensor) -> None:
        """residual += allreduce(a @ W^T); out = rmsnorm(residual) * norm_w, with W's two column halves pipelined
        against their all-reduces (TP_OVERLAP above): half 0 reduced on the side stream into a persistent buffer,
        half 1 reduced + joined + residual + RMSNorm in one fused launch."""
        car = pstate.custom_ar()
        side, (ev_in, ev1, ev_done) = _overlap_stream(a.device)
        main = torch.cuda.current_stream(a.device)
        nb = wt.shape[0] // 2
        T = a.shape[0]
        key = (a.device, T, nb * 32)
        h0 = _OVL.get(key)
        if h0 is None:  # persistent (a graph capture records a fixed address; stream order keeps uses apart)
            h0 = _OVL[key] = torch.empty(T, nb * 32, dtype=self.dtype, device=a.device)
        y0 = ops.linear_stream(a, wt[:nb])
        ev_in.record(main)
        with torch.cuda.stream(side):
            side.wait_event(ev_in)
            car.all_reduce(y0, out=h0)  # overlaps the second half's GEMM below
            ev_done.record(side)
        y1 = ops.linear_stream(a, wt[nb:])
        main.wait_event(ev_done)  # joined: half 0 is reduced (and every buffer the side stream read is released)
        car.all_reduce_add_rmsnorm(y1, residual, norm_w, eps, out, pre=h0)

    def _embed(self, tokens: torch.Tensor) -> torch.Tensor:
        if self.tp == 1:
            return F.embedding(tokens, self.embed)
        lo = self.tp_rank * self.vocab_local
        local = tokens - lo
        mask = (local < 0) | (local >= self.vocab_local)
        h = F.embedding(local.clamp(0, self.vocab_local - 1), self.embed)
        h = h.masked_fill(mask[:, None], 0)
        return pstate.tp_all_reduce(h)

    # ------------------------------------------------------------------------------------------------------------
    def weight_bytes(self) -> int:
        """Device bytes of every weight tensor, wave-tiled copies included (so tiled-only models report fully)."""
        ts = list(self.named_tensors().values()) + [self.lm_head_t]
        ts += [getattr(lw, s) for lw in self.layers for s in LayerWeights.__slots__ if s.endswith("_t")]
        return sum(t.numel() * t.element_size() for t in ts if isinstance(t, torch.Tensor))

    def named_tensors(self) -> dict[str, torch.Tensor]:
        out = {"embed": self.embed, "lm_head": self.lm_head, "final_norm": self.final_norm}
        for i, lw in enumerate(self.layers):
            for s in LayerWeights.__slots__:
                t = getattr(lw, s)
                if isinstance(t, torch.Tensor) and not s.endswith("_t"):
                    out[f"layers.{i}.{s}"] = t
        return {k: v for k, v in out.items() if v is not None}
