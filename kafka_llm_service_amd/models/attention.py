"""Paged attention for one engine step (mixed decode + chunked-prefill batch), dispatched to the CDNA4 kernels.

Token layout of a step: rows [0, B) are the B decode tokens (one per running sequence), rows [B, T) are prefill
chunk tokens. Per layer:
  * decode rows: split-K paged decode (``attn_decode``) writes (O, lse) partials, ``attn_merge`` combines them.
    When all decode sequences share the same first P KV pages (the ~18k-token Kafka system prompt, SURVEY.md §0,
    §7.4 #1) the step runs CASCADE attention: the shared prefix is attended once for all B sequences by the MFMA
    tile kernel (``attn_prefill`` with the decode tokens as query rows, prefix split into key chunks), the
    per-thread suffix by the decode kernel from ``kv_start = P``; everything merges by log-sum-exp.
  * prefill rows: work items of up to 128 (token, head) rows against the causal key range (``attn_prefill``)
    write bf16 output directly.

``AttnMeta`` holds only device tensors that the model runner prepares once per step (shared by all layers), so
the decode path is hipGraph-capturable (fixed shapes per batch bucket).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from kafka_llm_service_amd import ops


@dataclass
class AttnMeta:
    num_decode: int = 0                  # B
    num_tokens: int = 0                  # T
    block_tables: torch.Tensor | None = None   # int32 [rows, max_blocks]; rows [0,B) decode seqs, then prefill seqs
    # decode
    seq_lens: torch.Tensor | None = None       # int32 [B]  (KV length incl. the new token)
    kv_start: torch.Tensor | None = None       # int32 [B]  (cascade: P, else None)
    num_splits: int = 1                        # decode split-K factor over the suffix
    prefix_items: torch.Tensor | None = None   # int32 [n, 8] cascade prefix work items (rows = decode tokens)
    num_prefix_splits: int = 0
    part: torch.Tensor | None = None           # f32 [B, Hq, S_total, D]
    lse: torch.Tensor | None = None            # f32 [B, Hq, S_total]
    # prefill
    prefill_items: torch.Tensor | None = None  # int32 [m, 8] (q_start relative to row B)
    q_limit: torch.Tensor | None = None        # int32 [T] absolute causal limit per query token
    # long-context prefill with few query tiles: items are split along the key range (flash-decoding style) into
    # partials [T - B, Hq, prefill_splits, D] merged by log-sum-exp
    prefill_splits: int = 0
    prefill_part: torch.Tensor | None = None
    prefill_lse: torch.Tensor | None = None
    scale: float = 1.0
    extra: dict = field(default_factory=dict)

    @property
    def s_total(self) -> int:
        return self.num_prefix_splits + self.num_splits


_OVERLAP = os.environ.get("KAFKA_ATTN_OVERLAP", "0") == "1"
_SIDE: dict = {}


def _side_stream(dev: torch.device):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, meta: AttnMeta,
                    out: torch.Tensor) -> torch.Tensor:
    """q [T, Hq, D] (post-RoPE) -> out [T, Hq, D] bf16.

    With ``KAFKA_ATTN_OVERLAP=1`` the cascade prefix pass (MFMA tile kernel, compute-heavy) runs on a side HIP stream
    concurrently with the suffix decode pass (HBM-bound); both write disjoint split slots of the same partials and the
    merge waits for both (fork/join with events; hipGraph-capturable). Off by default until measured."""
    B = meta.num_decode
    if B > 0:
        qd = q[:B]
        overlap = _OVERLAP and q.is_cuda and meta.prefix_items is not None
        if overlap:
            main = torch.cuda.current_stream(q.device)
            side = _side_stream(q.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                ops.attn_prefill(meta.prefix_items, qd, k_cache, v_cache, meta.block_tables, meta.q_limit,
                                 meta.scale, out_part=meta.part, lse_part=meta.lse)
        elif meta.prefix_items is not None:
            ops.attn_prefill(meta.prefix_items, qd, k_cache, v_cache, meta.block_tables, meta.q_limit,
                             meta.scale, out_part=meta.part, lse_part=meta.lse)
        # the decode kernel merges the prefix partials itself and writes the final rows (one split per sequence —
        # the usual case at 64+ sequences — directly, several through its ticket counters); else merge kernel
        fused = meta.num_splits + meta.num_prefix_splits <= 64 and not overlap
        ops.attn_decode(qd, k_cache, v_cache, meta.block_tables, meta.seq_lens, meta.kv_start, meta.part,
                        meta.lse, meta.num_splits, meta.num_prefix_splits, meta.scale, out=out[:B] if fused else None)
        if overlap:
            main.wait_stream(side)
        if not fused:
            ops.attn_merge(meta.part, meta.lse, out[:B])
    if meta.prefill_items is not None and meta.num_tokens > B:
        if meta.prefill_splits:
            ops.attn_prefill(meta.prefill_items, q[B:], k_cache, v_cache, meta.block_tables, meta.q_limit[B:],
                             meta.scale, out_part=meta.prefill_part, lse_part=meta.prefill_lse)
            ops.attn_merge(meta.prefill_part, meta.prefill_lse, out[B:])
        else:
            ops.attn_prefill(meta.prefill_items, q[B:], k_cache, v_cache, meta.block_tables, meta.q_limit[B:],
                             meta.scale, out=out[B:])
    return out


def default_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
