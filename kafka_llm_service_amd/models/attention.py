"""Paged attention for one engine step (mixed decode + chunked-prefill batch), dispatched to the CDNA4 kernels.

Token layout of a step: rows [0, B) are the B decode tokens (one per running sequence), rows [B, T) are prefill
chunk tokens. Per layer:
  * decode rows: the decode kernel (``attn_decode_items``) streams each row's KV in work items of about equal size
    (a long history is split into pieces whose partials the last piece merges through ticket counters).
    CASCADE: decode rows that share their first P KV pages (the ~18k-token Kafka system prompt, SURVEY.md §0, §7.4
    #1) form a prefix group; each group's prefix is attended ONCE for all its rows by the MFMA tile kernel
    (``attn_prefill`` with the decode tokens as query rows, the prefix split into key chunks) and the decode kernel
    covers only the per-row suffix [P, len), folding the prefix partials into its merge. Rows with different system
    prompts form different groups (model_runner.prefix_groups); rows without a group read their whole context.
  * prefill rows: work items of up to 256 (token, head) rows against the causal key range (``attn_prefill``)
    write bf16 output directly, or (long ranges) fp32 partials merged by ``attn_merge``. A new turn behind a cascade
    group's prefix rides in the group's prefix pass twice over: its prefix pieces and its own keys' pieces are items
    of the same launch (model_runner.build_host ``join_suffix``), leaving only the merge.

``AttnMeta`` holds only device tensors that the model runner prepares once per step (shared by all layers), so
the decode path is hipGraph-capturable (fixed shapes per batch bucket).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import torch

from kafka_llm_service_amd import ops

# KAFKA_FUSED_PREFILL_MERGE=0: prefill rows' partials merged by their own attn_merge launch, never by the decode launch
FUSE_PREFILL_MERGE = os.environ.get("KAFKA_FUSED_PREFILL_MERGE", "1") == "1"


@dataclass
class AttnMeta:
    num_decode: int = 0                  # B
    num_tokens: int = 0                  # T
    block_tables: torch.Tensor | None = None   # int32 [rows, W]; rows [0,B) decode seqs, then prefill seqs
    # decode
    decode_items: torch.Tensor | None = None   # int32 [n, 8] (b, lo, hi, split, nsplit, npre, 0, 0)
    prefix_items: torch.Tensor | None = None   # int32 [m, 8] cascade prefix work items (rows = decode tokens)
    s_total: int = 1                           # partial slots per decode row
    part: torch.Tensor | None = None           # f32 [B, Hq, s_total, D]
    pre_part: torch.Tensor | None = None       # bf16, part's shape: the tile-v3 cascade's prefix partials
    lse: torch.Tensor | None = None            # f32 [B, Hq, s_total]
    # prefill
    prefill_items: torch.Tensor | None = None  # int32 [m, 8] (q_start relative to row B)
    q_limit: torch.Tensor | None = None        # int32 [T] absolute causal limit per query token
    # long prefill tiles are split along the key range (flash-decoding style) into partials
    # [T - B, Hq, prefill_splits, D] merged by log-sum-exp over ``prefill_merge``; the other tiles write rows directly
    prefill_splits: int = 0
    prefill_part: torch.Tensor | None = None
    prefill_lse: torch.Tensor | None = None
    prefill_merge: list = field(default_factory=list)  # (lo, hi) prefill row ranges of split tiles
    prefix_joined: bool = False                # prefill rows take part in the cascade prefix pass (alt partials)
    scale: float = 1.0
    variant: int = 0                           # tile-kernel variant (ops.tile_rows): 0 = 8 waves / 256 rows
    extra: dict = field(default_factory=dict)


def _prefill_part(q, k_cache, v_cache, meta: AttnMeta, out: torch.Tensor) -> None:
    B = meta.num_decode
    if meta.prefill_items is not None:  # (None when every prefill tile rode in the cascade launch)
        split = bool(meta.prefill_splits)
        ops.attn_prefill(meta.prefill_items, q[B:], k_cache, v_cache, meta.block_tables, meta.q_limit[B:],
                         meta.scale, out=out[B:], out_part=meta.prefill_part if split else None,
                         lse_part=meta.prefill_lse if split else None, variant=meta.variant)
    for lo, hi in meta.prefill_merge:
        ops.attn_merge(meta.prefill_part[lo:hi], meta.prefill_lse[lo:hi], out[B + lo:B + hi])


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, meta: AttnMeta,
                    out: torch.Tensor) -> None:
    """q [T, Hq, D] (post-RoPE) -> out [T, Hq, D] bf16."""
    B = meta.num_decode
    if B > 0:
        qd = q[:B]
        if meta.prefix_items is not None:
            # new-turn prefill rows that share the prefix ride along (items flagged alt: fp32 partials in their own
            # merge buffer, model_runner.build_host); the kernel reads only the q rows its items name
            joined = meta.prefix_joined and meta.prefill_part is not None
            ops.attn_prefill(meta.prefix_items, q if joined else qd, k_cache, v_cache, meta.block_tables,
                             meta.q_limit, meta.scale,
                             out_part=meta.pre_part if meta.pre_part is not None else meta.part, lse_part=meta.lse,
                             variant=meta.variant, alt_part=meta.prefill_part if joined else None,
                             alt_lse=meta.prefill_lse if joined else None, alt_tok_off=B)
        # the decode kernel merges each row's prefix partials and its own pieces and writes the final rows; when
        # every prefill tile rode in the cascade launch, its extra workgroups also merge the prefill rows' partials
        merge = None
        if meta.prefill_items is None and len(meta.prefill_merge) == 1 and FUSE_PREFILL_MERGE:
            lo, hi = meta.prefill_merge[0]
            merge = (meta.prefill_part[lo:hi], meta.prefill_lse[lo:hi], out[B + lo:B + hi])
        ops.attn_decode_items(qd, k_cache, v_cache, meta.block_tables, meta.decode_items, meta.part, meta.lse,
                              meta.scale, out=out[:B], pre_part=meta.pre_part, merge=merge)
        if merge is not None:
            return
    if meta.num_tokens > B and (meta.prefill_items is not None or meta.prefill_merge):
        _prefill_part(q, k_cache, v_cache, meta, out)


def default_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)
