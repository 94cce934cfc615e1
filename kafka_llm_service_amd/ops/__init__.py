"""Public op API. GPU tensors run the hand-written CDNA4 HIP kernels (``csrc/*.hip``) and nothing else;
CPU tensors run the fp32 PyTorch references in ``reference.py`` (unit tests / CPU-only tooling).

Kernel inventory:
  rmsnorm / fused_add_rmsnorm / silu_mul        csrc/norm_act.hip
  rope_kv_write (RoPE + paged KV write)         csrc/rope_kv.hip
  attn_decode / attn_prefill / attn_merge       csrc/attention.hip   (MFMA 32x32x16 bf16, paged, split-K, cascade)
  sample (greedy / temperature / top-k / top-p) csrc/sampling.hip
  moe_* / grouped GEMM                          csrc/moe.hip
  custom all-reduce                             csrc/allreduce.hip
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import reference as ref
from ._ext import ext

PAGE = ref.PAGE
kv_cache_shapes = ref.kv_cache_shapes
kv_page_bytes = ref.kv_page_bytes
is_fp8_cache = ref.is_fp8_cache


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def is_slab(t: torch.Tensor) -> bool:
    """Split-K partial sums of the decode GEMM: fp32 [S, T, n] (``linear_stream``). The slab-aware ops below
    (fused_add_rmsnorm, silu_mul, rope_kv_write) sum them while loading; ``slab_reduce`` gives the bf16 tensor."""
    return t.dtype == torch.float32 and t.dim() == 3


def rows_of(t: torch.Tensor) -> int:
    return t.shape[1] if is_slab(t) else t.shape[0]


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    if _gpu(x):
        ext().rmsnorm(out.view(-1, x.shape[-1]), x.reshape(-1, x.shape[-1]), w, float(eps))
    else:
        out.copy_(ref.rmsnorm(x, w, eps))
    return out


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                      out: torch.Tensor | None = None) -> torch.Tensor:
    """residual <- x + residual (in place); returns rmsnorm(residual) * w (into ``out`` or a new tensor).
    ``x`` may be a split-K slab [S, T, d] (summed in fp32 before the add)."""
    slab = is_slab(x)
    if out is None:
        out = torch.empty(residual.shape, dtype=residual.dtype, device=x.device)
    if _gpu(x):
        xa = x if slab else x.reshape(-1, x.shape[-1])
        ext().fused_add_rmsnorm(out.view(-1, x.shape[-1]), xa, residual.view(-1, x.shape[-1]), w, float(eps))
    else:
        y, s = ref.fused_add_rmsnorm(x.sum(0) if slab else x, residual, w, eps)
        residual.copy_(s)
        out.copy_(y)
    return out


def silu_mul(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """silu(x[..., :F]) * x[..., F:] (bf16 out); ``x`` may be a split-K slab [S, T, 2F]."""
    F = x.shape[-1] // 2
    slab = is_slab(x)
    if out is None:
        lead = (x.shape[1],) if slab else x.shape[:-1]
        out = torch.empty(*lead, F, dtype=torch.bfloat16 if slab else x.dtype, device=x.device)
    if _gpu(x):
        ext().silu_mul(out.view(-1, F), x if slab else x.reshape(-1, 2 * F))
    else:
        out.copy_(ref.silu_mul(x.sum(0) if slab else x))
    return out


def rope_kv_write(qkv, positions, cos_sin, q_out, k_cache, v_cache, slot_mapping, Hq: int, Hkv: int) -> None:
    """RoPE on q/k + paged KV write; ``qkv`` is bf16 [T, W] or a split-K slab [S, T, W]."""
    if _gpu(qkv):
        ext().rope_kv_write(qkv, positions, cos_sin, q_out, k_cache, v_cache, slot_mapping, int(Hq), int(Hkv))
    else:
        ref.rope_kv_write(qkv.sum(0) if is_slab(qkv) else qkv, positions, cos_sin, q_out, k_cache, v_cache,
                          slot_mapping, Hq, Hkv)


_TICKETS: dict = {}


def _tickets(dev: torch.device, n: int, pool: str = "decode") -> torch.Tensor:
    """Zeroed int32 counters for a kernel's ticket merge (re-armed by the kernel itself, so one buffer per device and
    pool serves every layer and step; allocated once, large, so graph capture never allocates). Pool "decode":
    decode attention, per row x kv head."""
    t = _TICKETS.get((dev, pool))
    if t is None or t.numel() < n:
        t = _TICKETS[(dev, pool)] = torch.zeros(max(n, 1 << 16), dtype=torch.int32, device=dev)
    return t


DECODE_ITEM = 8  # int32 fields of a decode work item: (b, lo, hi, split, nsplit, npre, 0, 0)


def attn_decode_items(q, k_cache, v_cache, block_tables, items, out_part, lse_part, scale: float, out=None,
                      pre_part=None, merge=None) -> None:
    """Paged decode attention over work items (int32 [n, 8]: row b, key range [lo, hi), piece ``split`` of
    ``nsplit``, ``npre`` prefix partials in front). Each item writes its (O, lse2) partial to slot npre + split of
    [B, Hq, S_total, D]; with ``out`` (npre + nsplit <= 64 per row) the rows are instead merged with their prefix
    partials and written as final bf16 — a one-piece row directly, a split row by the last piece to finish (ticket
    counters, no merge kernel). ``pre_part``: bf16 prefix partials written by the tile-v3 cascade (slots < npre,
    out_part's shape) — half the bytes of the fp32 round trip. ``merge`` = (part [rows, Hq, S2, D], lse [rows, Hq,
    S2], out [rows, Hq, D]): other rows' fp32 partials (a step's prefill rows) merged into ``out`` by extra
    workgroups of the same launch, as ``attn_merge`` would."""
    if _gpu(q):
        tk = _tickets(q.device, q.shape[0] * k_cache.shape[1]) if out is not None else None
        mp, ml, mo = merge if merge is not None else (None, None, None)
        ext().attn_decode(q, k_cache, v_cache, block_tables, items, out_part, lse_part, float(scale), out, tk,
                          pre_part, mp, ml, mo)
        return
    ref.attn_decode_items(q, k_cache, v_cache, block_tables, items, out_part, lse_part, scale, out, pre_part)
    if merge is not None:
        ref.attn_merge(*merge)


def uniform_decode_items(seq_lens: torch.Tensor, kv_start: torch.Tensor | None, num_splits: int,
                         split_offset: int) -> torch.Tensor:
    """Decode items splitting every row's keys [kv_start, seq_len) into ``num_splits`` 32-key-aligned pieces, with
    partial slots from ``split_offset`` (built on the tensors' device, no host sync)."""
    B, S = seq_lens.numel(), int(num_splits)
    dev = seq_lens.device
    L = seq_lens.long()
    st = kv_start.long()[:B] if kv_start is not None else torch.zeros_like(L)
    a0 = st - st % 32
    nb = ((L - a0 + 31) // 32).clamp(min=0)
    bps = (nb + S - 1) // S
    b = torch.arange(B, device=dev).repeat_interleave(S)
    s = torch.arange(S, device=dev).repeat(B)
    blo = s * bps[b]
    bhi = torch.minimum(nb[b], blo + bps[b])
    lo = torch.maximum(st[b], a0[b] + blo * 32)
    hi = torch.maximum(lo, torch.minimum(L[b], a0[b] + bhi * 32))
    z = torch.zeros_like(b)
    return torch.stack([b, lo, hi, s, z + S, z + int(split_offset), z, z], 1).to(torch.int32).contiguous()


def attn_decode(q, k_cache, v_cache, block_tables, seq_lens, kv_start, out_part, lse_part, num_splits: int,
                split_offset: int, scale: float, out=None) -> None:
    """Uniform split-K decode (every row's keys [kv_start, seq_len) in ``num_splits`` pieces) on the work-item
    kernel: partials at slots [split_offset, split_offset + num_splits), or with ``out`` merged with the prefix
    partials [0, split_offset) into final bf16 rows (see ``attn_decode_items``)."""
    if out is not None and split_offset + num_splits > 64:
        raise ValueError("fused-merge decode needs <= 64 partials")
    items = uniform_decode_items(seq_lens[:q.shape[0]], kv_start, num_splits, split_offset)
    attn_decode_items(q, k_cache, v_cache, block_tables, items, out_part, lse_part, scale, out)


def attn_prefill(items, q, k_cache, v_cache, block_tables, q_limit, scale: float, out=None, out_part=None,
                 lse_part=None, variant: int = 0, alt_part=None, alt_lse=None, alt_tok_off: int = 0) -> None:
    """Work-item paged attention (chunked prefill / cascade prefix). ``items`` is int32 [n, 8]:
    (q_start, q_count, bt_row, kv_lo, kv_hi, split, alt, 0). Items with ``alt`` set (tile variant 3) write their
    partial into ``alt_part`` / ``alt_lse`` (fp32 [rows, Hq, S2, D], row = token - ``alt_tok_off``) instead of
    ``out_part``: the cascade's prefix pass over a step's new-turn prefill rows."""
    if _gpu(q):
        ext().attn_prefill(items, q, k_cache, v_cache, block_tables, q_limit, out, out_part, lse_part, float(scale),
                           int(variant), alt_part, alt_lse, int(alt_tok_off))
    else:
        ref.attn_prefill_items(items, q, k_cache, v_cache, block_tables, q_limit, scale, out, out_part, lse_part,
                               alt_part, alt_lse, alt_tok_off)


def tile_rows(variant: int = 0) -> int:
    """Query rows ((token, head) pairs of one KV head) per attn_prefill work item for a kernel variant."""
    return 256 if variant in (0, 3) else 128


def attn_merge(part, lse, out, lse_out=None, pre=None, npre: int = 0) -> None:
    """Log-sum-exp merge of the S partials per (row, head) of part f32 [rows, Hq, S, D] -> out bf16; with ``pre``
    (bf16, part's shape) slots [0, npre) are read from it (the cascade's prefix partials)."""
    if _gpu(part):
        ext().attn_merge(part, lse, out, lse_out, pre, int(npre))
    else:
        ref.attn_merge(part, lse, out, lse_out, pre, npre)


_SAMPLE_WS: dict = {}
_SAMPLE_SPLIT = int(__import__("os").environ.get("KAFKA_SAMPLE_SPLIT", "8"))


def _sample_ws(dev: torch.device, n: int) -> torch.Tensor:
    """Sampler workspace: 65536 zeroed per-row tickets (re-armed by the kernel) + split winners; allocated once per
    device, large enough for graph capture never to allocate."""
    t = _SAMPLE_WS.get(dev)
    if t is None or t.numel() < n:
        t = _SAMPLE_WS[dev] = torch.zeros(max(n, 65536 + 2 * 4096 * 8), dtype=torch.int32, device=dev)
    return t


def sample(logits, temperature=None, top_p=None, top_k=None, seeds=None, step=None, out=None, proc=None,
           mask_tab=None, counts=None) -> torch.Tensor:
    """Sampled ids [B] (int64). ``proc`` int32 [B, 8] turns on the per-row logits processing of the kernel (grammar
    bitmask rows of ``mask_tab``, forced ids, presence / frequency penalties from ``counts``, which the sampler
    updates with every drawn token; engine/logits_proc.py builds all three)."""
    B = logits.shape[0]
    if out is None:
        out = torch.empty(B, dtype=torch.long, device=logits.device)
    if _gpu(logits):
        V = logits.shape[1]
        nsplit = _SAMPLE_SPLIT if V >= 16384 else 1  # a row over 8 workgroups (greedy / plain temperature)
        ws = _sample_ws(logits.device, 65536 + 2 * B * nsplit) if nsplit > 1 else None
        ext().sample(logits, temperature, top_p, top_k, seeds, step, out, ws, nsplit, proc, mask_tab, counts)
    else:
        ref.sample(logits, temperature, top_p, top_k, seeds, step, out, proc, mask_tab, counts)
    return out


def tile_weight(w: torch.Tensor, glu: bool = False) -> torch.Tensor:
    """Row-major weight [N, K] -> the wave-tiled layout [N/32, K/16, 64, 8] read by the weight-streaming decode GEMM
    (csrc/wstream_gemm.hip): lane l = (r = l % 32, h = l // 32) of tile (nb, kb) holds W[32 nb + r, 16 kb + 8 h : +8].
    ``glu``: W = [gate; up] (N = 2F); the 32-row tiles are interleaved gate_0, up_0, gate_1, up_1, ... so one
    workgroup holds matching gate/up columns and the GEMM can emit silu(gate) * up directly."""
    N, K = w.shape
    t = w.reshape(N // 32, 32, K // 16, 2, 8).permute(0, 2, 3, 1, 4)
    if glu:
        t = t.reshape(2, N // 64, K // 16, 2, 32, 8).transpose(0, 1)
    return t.contiguous().view(N // 32, K // 16, 64, 8)


def untile_weight(wt: torch.Tensor, glu: bool = False) -> torch.Tensor:
    nb, kb = wt.shape[0], wt.shape[1]
    if glu:
        wt = wt.view(nb // 2, 2, kb, 64, 8).transpose(0, 1).reshape(nb, kb, 64, 8)
    return wt.reshape(nb, kb, 2, 32, 8).permute(0, 3, 1, 2, 4).reshape(nb * 32, kb * 16)


# Steps of up to this many rows run the dense projections on the weight-streaming kernel (csrc/wstream_gemm.hip).
# The kernel takes up to 256 rows: one 192-row tile (MT = 6) up to 192, beyond that two row tiles of 128 sharing each
# weight slice through the MALL, where it loses to hipBLASLt (gate_up 101 vs 66 us at 168..248 rows; bench 7,359 vs
# 7,546 tok/s, profiles/r02/stream_max_m_256_rejected.jsonl). The 192-row tile only ties the skinny GEMM + hipBLASLt
# path of 129..192-row steps (8,725 vs 8,732 tok/s, profiles/r06/mt6/), so the default stays 128; tiled-only models
# (no row-major copy for hipBLASLt) stream every step up to 256 rows. Env KAFKA_STREAM_MAX_M (1..256).
STREAM_MAX_M = max(1, min(256, int(os.environ.get("KAFKA_STREAM_MAX_M", "128"))))
STREAM_KERNEL_MAX_M = 256


def stream_plan(M: int, N: int, K: int, max_splits: int = 8) -> tuple[int, int, int] | None:
    """(row tiles, K chunk, splits) of the decode GEMM for a shape, None if unsupported (same rule as
    kafka_wstream_plan in csrc/wstream_gemm.hip, mirrored so CPU runs take the same split decisions)."""
    if M < 1 or M > STREAM_KERNEL_MAX_M or N % 32 or N <= 0:
        return None
    mt = 1 if M <= 32 else (2 if M <= 64 else (3 if M <= 96 else (4 if M <= 128 or M > 192 else 6)))
    kc = 128 if mt >= 4 else 256
    if K % kc or K <= 0:
        return None
    nx, chunks, s = (N + 127) // 128 * ((M + 32 * mt - 1) // (32 * mt)), K // kc, 1
    target = 192
    while s * 2 <= max_splits and s * 2 <= 8 and chunks % (s * 2) == 0 and nx * s < target:
        s *= 2
    return mt, kc, s


SKINNY_MIN_M, SKINNY_MAX_M = 129, 256


def skinny_plan(M: int, N: int, K: int, max_splits: int = 8) -> int:
    """Splits of the skinny GEMM (csrc/skinny_gemm.hip kafka_skinny_plan, mirrored for CPU runs); 0 = unsupported."""
    if M < SKINNY_MIN_M or M > SKINNY_MAX_M or N % 128 or K % 64:
        return 0
    nx, s = N // 128, 1
    while s * 2 <= max_splits and nx * s < 192 and K % (64 * s * 2) == 0 and K // (s * 2) >= 256:
        s *= 2
    return s


def linear_skinny(x: torch.Tensor, wt: torch.Tensor, max_splits: int = 8, glu: bool = False) -> torch.Tensor:
    """y = x @ W^T for 129..256 rows from the wave-tiled weight (mixed decode + prefill steps): bf16 [M, N] (or the
    activated [M, N/2] with ``glu``) for one split, else fp32 split-K slabs [S, M, N] in gate | up order for glu."""
    M, K = x.shape
    N = wt.shape[0] * 32
    S = skinny_plan(M, N, K, max_splits)
    if S == 0:
        raise ValueError(f"linear_skinny: unsupported shape M={M} N={N} K={K}")
    if _gpu(x):
        if S == 1:
            y = torch.empty(M, N // 2 if glu else N, dtype=x.dtype, device=x.device)
            ext().skinny_gemm(x, wt, y, None, 1, bool(glu))
            return y
        p = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        ext().skinny_gemm(x, wt, None, p, int(S), bool(glu))
        return p
    w = untile_weight(wt, glu).float()
    y = x.float() @ w.t()
    if S == 1:
        return (ref.silu_mul(y) if glu else y).to(x.dtype)
    p = torch.zeros(S, M, N, dtype=torch.float32)
    p[0] = y
    return p


def linear_stream(x: torch.Tensor, wt: torch.Tensor, max_splits: int = 8, nt: bool = True,
                  glu: bool = False) -> torch.Tensor:
    """y = x @ W^T for decode-sized M (<= 128) from the wave-tiled weight ``wt``: the weight-streaming MFMA kernel.
    Returns bf16 [M, N] when the plan has one split, else the fp32 split-K slabs [S, M, N] (a slab; the consumer
    kernels sum it while loading). ``glu`` (wt tiled with glu=True): a one-split plan returns the ACTIVATED
    silu(gate) * up [M, N/2] (fused epilogue); a split plan returns gate | up slabs as usual (see ``linear_glu``)."""
    M, K = x.shape
    N = wt.shape[0] * 32
    plan = stream_plan(M, N, K, max_splits)
    if plan is None:
        raise ValueError(f"linear_stream: unsupported shape M={M} N={N} K={K}")
    S = plan[2]
    if _gpu(x):
        if S == 1:
            y = torch.empty(M, N // 2 if glu else N, dtype=x.dtype, device=x.device)
            ext().wstream_gemm(x, wt, y, None, int(max_splits), bool(nt), bool(glu))
            return y
        p = torch.empty(S, M, N, dtype=torch.float32, device=x.device)
        ext().wstream_gemm(x, wt, None, p, int(max_splits), bool(nt), bool(glu))
        return p
    w = untile_weight(wt, glu).float()
    xf = x.float()
    if S == 1:
        y = xf @ w.t()
        if glu:
            return ref.silu_mul(y).to(x.dtype)
        return y.to(x.dtype)
    ks = K // S
    return torch.stack([xf[:, s * ks:(s + 1) * ks] @ w[:, s * ks:(s + 1) * ks].t() for s in range(S)])


def linear_glu(x: torch.Tensor, wt: torch.Tensor, max_splits: int = 8) -> torch.Tensor:
    """silu(x @ Wg^T) * (x @ Wu^T) from GLU-tiled gate_up weights: fused into the GEMM epilogue when the plan has one
    split, else the GEMM's slabs go through silu_mul."""
    N = wt.shape[0] * 32
    plan = stream_plan(x.shape[0], N, x.shape[1], max_splits)
    y = linear_stream(x, wt, max_splits, glu=True)
    return y if plan is not None and plan[2] == 1 else silu_mul(y)


# ---- fused decode layer (csrc/wstream_gemm.hip FIN_*): deferred RMSNorm + split-K finishers ----------------------
# A decode layer runs as qkv(+RoPE/KV write) -> attention -> o(+residual add, next norm) -> gate_up(+row scale,
# SwiGLU) -> down(+residual add, next norm): the RMSNorm and RoPE kernels leave the step. The residual producer writes
# X' = bf16(h * w) and per-128-column partial sums of h^2 (``ss`` fp32 [d/128, T]); the consumer GEMM scales each
# output row by r = rsqrt(sum(ss) / d + eps) — rmsnorm(h) . W^T = r * ((h * w) . W^T).

def fin_row_scale(ss: torch.Tensor | None, M: int, d: int, eps: float) -> torch.Tensor | None:
    """r[m] = rsqrt(sum_j ss[j, m] / d + eps) (fp32 [M]) — the deferred RMSNorm scale; None without partials."""
    if ss is None:
        return None
    return torch.rsqrt(ss[:, :M].float().sum(0) / d + eps)


FIN_POOLS = ("fin", "fin_o", "fin_down", "fin_qkv")


def fin_errors(dev: torch.device) -> int:
    """Error words of the fused GEMM finishers (the last int of each ticket pool; csrc FinArgs::err): nonzero if a
    finisher ran on another XCD than the splits that kept their slabs in their home L2 — the result of that launch is
    unreliable. Checked by the tests, smoke() and the bench (a host sync: not for the hot path)."""
    n = 0
    for pool in FIN_POOLS:
        t = _TICKETS.get((dev, pool))
        if t is not None:
            n |= int(t[-1].item())
    return n


# KAFKA_FIN_STAMPS=<file.json>: every fused GEMM launch records per-workgroup phase stamps (csrc FinArgs::stamps) and
# the anatomy of the last launches per kind is written to that file at exit (benchmarks/fused_bench.py reads the same
# stamps in isolation; this is the in-engine view)
_FIN_STAMPS = os.environ.get("KAFKA_FIN_STAMPS")
_STAMP_LOG: list = []


def _stamps_for(kind: str, grid: int, dev: torch.device):
    if not _FIN_STAMPS:
        return None
    if not _STAMP_LOG:
        import atexit
        atexit.register(_dump_stamps)
    t = torch.zeros(grid * 8 + 8, dtype=torch.long, device=dev)
    _STAMP_LOG.append((kind, grid, t))
    del _STAMP_LOG[:-2000]
    return t


def _dump_stamps() -> None:
    import json
    import statistics
    out: dict = {}
    for kind, grid, t in _STAMP_LOG:
        a = t[:grid * 8].view(grid, 8).cpu().double() / 100.0
        a = a - a[:, 0].min()
        fin = a[:, 4] > 0
        rec = {"loop_max": float((a[:, 1] - a[:, 0]).max()), "last_loop_end": float(a[:, 1].max()),
               "first_start_to_last_start": float(a[:, 0].max())}
        if fin.any():
            rec.update(end=float(a[fin, 4].max()), tail=float(a[fin, 4].max() - a[:, 1].max()),
                       fin_med=float((a[fin, 4] - a[fin, 3]).median()),
                       drain_med=float((a[a[:, 2] > 0, 2] - a[a[:, 2] > 0, 1]).median()) if (a[:, 2] > 0).any() else 0.0,
                       ticket_med=float((a[fin, 3] - a[fin, 2]).median()))
        out.setdefault(f"{kind}/grid{grid}", []).append(rec)
    summary = {k: {f: round(statistics.median(r[f] for r in v if f in r), 2) for f in v[-1]} | {"calls": len(v)}
               for k, v in out.items()}
    with open(_FIN_STAMPS, "w") as f:
        json.dump(summary, f, indent=1)


def _fin_scratch(x: torch.Tensor, N: int, max_splits: int) -> tuple[int, torch.Tensor | None]:
    M, K = x.shape
    plan = stream_plan(M, N, K, max_splits)
    if plan is None or M > 128 or N % 128:
        raise ValueError(f"fused decode GEMM: unsupported shape M={M} N={N} K={K}")
    S = plan[2]
    return S, (torch.empty(S, M, N, dtype=torch.float32, device=x.device) if S > 1 else None)


def linear_res(x: torch.Tensor, wt: torch.Tensor, resid: torch.Tensor, nw: torch.Tensor, xn: torch.Tensor,
               ss_out: torch.Tensor, max_splits: int = 8, pool: str = "fin") -> None:
    """resid <- bf16(resid + x @ W^T) in place; xn <- bf16(resid * nw); ss_out[cb, m] = sum of resid[m, 128 cb:+128]^2
    (the o / down projection with the residual add and the next RMSNorm's producer half, csrc FIN_RES)."""
    N = wt.shape[0] * 32
    if _gpu(x):
        S, p = _fin_scratch(x, N, max_splits)
        ext().wstream_fin(1, x, wt, None, p, _tickets(x.device, N // 128 + 1, pool), None, 0.0, resid, nw, xn, ss_out,
                          None, None, None, None, None, None, 0, 0, int(max_splits),
                          _stamps_for(pool, N // 128 * S, x.device))
        return
    M = x.shape[0]
    y = x.float() @ untile_weight(wt).float().t()
    s = (resid.float() + y).to(resid.dtype)
    resid.copy_(s)
    xn.copy_((s.float() * nw.float()).to(xn.dtype))
    ss_out[:, :M] = s.float().pow(2).view(M, N // 128, 128).sum(-1).t()


def linear_qkv_rope(x: torch.Tensor, wt: torch.Tensor, ss_in: torch.Tensor | None, eps: float, positions, cos_sin,
                    q_out, k_cache, v_cache, slot_mapping, Hq: int, Hkv: int, max_splits: int = 8,
                    pool: str = "fin_qkv") -> None:
    """RoPE + paged KV write of r * (x @ Wqkv^T) (r: the deferred RMSNorm of x from ``ss_in``, or 1), in the QKV
    GEMM's split-K finisher (csrc FIN_ROPE); bf16 caches, head dim 128."""
    N = wt.shape[0] * 32
    M, K = x.shape
    if _gpu(x):
        S, p = _fin_scratch(x, N, max_splits)
        ext().wstream_fin(2, x, wt, None, p, _tickets(x.device, N // 128 + 1, pool), ss_in, float(eps), None, None,
                          None, None, positions, cos_sin, q_out, k_cache, v_cache, slot_mapping, int(Hq), int(Hkv),
                          int(max_splits), _stamps_for(pool, N // 128 * S, x.device))
        return
    y = x.float() @ untile_weight(wt).float().t()
    r = fin_row_scale(ss_in, M, K, eps)
    if r is not None:
        y = y * r[:, None]
    ref.rope_kv_write(y, positions, cos_sin, q_out, k_cache, v_cache, slot_mapping, Hq, Hkv)


def linear_glu_rs(x: torch.Tensor, wt: torch.Tensor, ss_in: torch.Tensor | None, eps: float) -> torch.Tensor:
    """silu(r g) * (r u) with [g | u] = x @ Wgu^T from GLU-tiled weights, one split (csrc FIN_GLU); r as above."""
    N = wt.shape[0] * 32
    M, K = x.shape
    if _gpu(x):
        y = torch.empty(M, N // 2, dtype=x.dtype, device=x.device)
        ext().wstream_fin(3, x, wt, y, None, _tickets(x.device, 1, "fin"), ss_in, float(eps), None, None, None, None,
                          None, None, None, None, None, None, 0, 0, 1, _stamps_for("glu", N // 128, x.device))
        return y
    y = x.float() @ untile_weight(wt, glu=True).float().t()
    r = fin_row_scale(ss_in, M, K, eps)
    if r is not None:
        y = y * r[:, None]
    F = N // 2
    return (torch.nn.functional.silu(y[:, :F]) * y[:, F:]).to(x.dtype)


def fin_supported(M: int, d: int, n_qkv: int, n_gu: int, head_dim: int, kw_gate_up: int = 2) -> bool:
    """Shapes the fused decode layer takes (else the model runs the unfused kernels): one row tile, 128-column heads,
    the gate_up row-scale partials fit its threads."""
    if not (1 <= M <= 128 and head_dim == 128 and d % 128 == 0 and d <= 4096 and n_qkv % 128 == 0 and
            n_gu % 128 == 0):
        return False
    if stream_plan(M, n_gu, d, 1) is None or stream_plan(M, n_qkv, d) is None or stream_plan(M, d, d) is None:
        return False
    mt, kc, _ = stream_plan(M, n_gu, d, 1)
    nth = 256 * (2 if mt == 2 and kc == 256 and d // kc >= 6 else 1)
    ssl, nss, tpr = 4096 // nth, d // 128, 1
    while tpr * ssl < nss:
        tpr *= 2
    return tpr <= 64 and M * tpr <= nth


def tile_experts(w: torch.Tensor, glu: bool = False) -> torch.Tensor:
    """Expert weights [E, N, K] -> wave-tiled [E, N/32, K/16, 64, 8] (``tile_weight`` per expert)."""
    E, N, K = w.shape
    out = torch.empty(E, N // 32, K // 16, 64, 8, dtype=w.dtype, device=w.device)
    for e in range(E):
        out[e].copy_(tile_weight(w[e], glu))
    return out


def untile_experts(wt: torch.Tensor, glu: bool = False) -> torch.Tensor:
    return torch.stack([untile_weight(wt[e], glu) for e in range(wt.shape[0])])


def stream_moe_supported(N: int, K: int) -> bool:
    return N % 64 == 0 and K % 256 == 0


# weight prefetch of the grouped streaming kernel pinned ahead of its MFMAs (as the dense one; toggled by
# benchmarks/moe_bench.py for its A/B)
GROUPED_PIN = True


def grouped_stream_glu(x: torch.Tensor, wt: torch.Tensor, r: "MoERouting", e_lo: int = 0) -> torch.Tensor:
    """silu(gate) * up for every routed (token, local expert) entry, rows in expert-sorted order [n_ent, F]: the
    weight-streaming grouped kernel on GLU-tiled expert weights (``tile_experts(w13, glu=True)``)."""
    T = x.shape[0]
    n_ent = r.perm_tok.numel()
    F = wt.shape[1] * 16
    y = torch.empty(n_ent, F, dtype=x.dtype, device=x.device)
    if _gpu(x):
        ext().wstream_grouped(x, wt, r.perm_tok, r.perm_w, r.expert_off, int(e_lo), int(T), True, y, None,
                              GROUPED_PIN)
        return y
    h = ref_grouped(x, untile_experts(wt, glu=True), r, e_lo, gather=True)
    y.copy_(ref.silu_mul(h))
    return y


def grouped_stream_combine(a: torch.Tensor, wt: torch.Tensor, r: "MoERouting", T: int, out: torch.Tensor,
                           e_lo: int = 0) -> torch.Tensor:
    """out[token] += w * (a[entry] @ W_e^T) over the local experts' entries (out f32 [T, N], zeroed by the caller)."""
    if _gpu(a):
        ext().wstream_grouped(a, wt, r.perm_tok, r.perm_w, r.expert_off, int(e_lo), int(T), False, None, out,
                              GROUPED_PIN)
        return out
    ref.grouped_gemm(a, untile_experts(wt), r.perm_tok, r.perm_w, r.expert_off, e_lo, False, None, out)
    return out


def ref_grouped(x, w, r, e_lo, gather):
    y = torch.zeros(r.perm_tok.numel(), w.shape[1], dtype=x.dtype)
    ref.grouped_gemm(x, w, r.perm_tok, r.perm_w, r.expert_off, e_lo, gather, y, None)
    return y


def slab_reduce(p: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [M, N] = sum of the split-K slabs [S, M, N] (bf16 inputs pass through)."""
    if not is_slab(p):
        return p
    if out is None:
        out = torch.empty(p.shape[1], p.shape[2], dtype=torch.bfloat16, device=p.device)
    if _gpu(p):
        ext().slab_reduce(p, out)
    else:
        out.copy_(p.sum(0))
    return out


rope_cos_sin = ref.rope_cos_sin


class MoERouting:
    """Device-side routing of one MoE layer (csrc/moe.hip ``moe_route``): everything the grouped GEMMs need."""
    __slots__ = ("topk_w", "topk_e", "perm_tok", "perm_w", "expert_off", "tile_off", "num_experts", "max_tiles")

    def __init__(self, topk_w, topk_e, perm_tok, perm_w, expert_off, tile_off, num_experts):
        self.topk_w, self.topk_e = topk_w, topk_e
        self.perm_tok, self.perm_w = perm_tok, perm_w
        self.expert_off, self.tile_off = expert_off, tile_off
        self.num_experts = num_experts
        self.max_tiles = (perm_tok.numel() + GG_BM - 1) // GG_BM + num_experts


GG_BM = 64  # row tile of the grouped GEMM (a routing bound the kernel and the host agree on)


def moe_route(logits: torch.Tensor, k: int) -> MoERouting:
    """softmax -> top-k -> renormalise, then a stable sort of the T*k entries by expert (token order inside)."""
    T, E = logits.shape
    dev = logits.device
    if _gpu(logits):
        tw = torch.empty(T, k, dtype=torch.float32, device=dev)
        te = torch.empty(T, k, dtype=torch.int32, device=dev)
        pt = torch.empty(T * k, dtype=torch.int32, device=dev)
        pw = torch.empty(T * k, dtype=torch.float32, device=dev)
        eo = torch.empty(E + 1, dtype=torch.int32, device=dev)
        to = torch.empty(E + 1, dtype=torch.int32, device=dev)
        ext().moe_route(logits, int(k), GG_BM, tw, te, pt, pw, eo, to)
        return MoERouting(tw, te, pt, pw, eo, to, E)
    tw, te, pt, pw, eo, to = ref.moe_route(logits, k, GG_BM)
    return MoERouting(tw, te, pt, pw, eo, to, E)


def grouped_gemm(x: torch.Tensor, w: torch.Tensor, r: MoERouting, gather: bool, e_lo: int = 0,
                 y: torch.Tensor | None = None, combine_out: torch.Tensor | None = None) -> torch.Tensor:
    """Per expert segment of the routed entries: Y = X_e . W_e^T (W = [E_local, N, K], experts [e_lo, e_lo+E_local)).

    gather=True reads A rows as x[perm_tok[r]] (token activations), else x[r] (expert-sorted rows).
    combine_out (f32 [T, N], zeroed by the caller) receives out[perm_tok[r]] += perm_w[r] * Y[r] instead of Y."""
    n_ent = r.perm_tok.numel()
    if combine_out is not None and combine_out.shape[0] != r.topk_w.shape[0]:
        raise ValueError("combine_out must have one row per routed token")
    if combine_out is None and y is None:
        y = torch.empty(n_ent, w.shape[1], dtype=x.dtype, device=x.device)
    if _gpu(x):
        ext().grouped_gemm(x, w, r.perm_tok, r.perm_w, r.expert_off, r.tile_off, int(e_lo), int(r.max_tiles),
                           bool(gather), y, combine_out)
    else:
        ref.grouped_gemm(x, w, r.perm_tok, r.perm_w, r.expert_off, e_lo, gather, y, combine_out)
    return combine_out if combine_out is not None else y


# ---- expert-parallel all-to-all (csrc/moe.hip ep_*, models/moe.py MoEBlock._a2a) --------------------------------
def ep_layout(T: int, ep: int, k: int, El: int, d: int) -> tuple[int, int, int]:
    """(owned tokens per rank Tl, slot capacity C per destination, metadata rows MR) of the EP send image
    [ep, C + MR, d]: a token's k experts are distinct, so at most min(k, El) of its pairs go to one rank."""
    Tl = max(1, -(-T // ep))
    C = Tl * min(k, El)
    MR = -(-(16 + 4 * C) // (2 * d))
    return Tl, C, MR


def ep_dispatch(x: torch.Tensor, topk_e: torch.Tensor, lo: int, n_own: int, El: int, ep: int, C: int,
                MR: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Send image [ep, C + MR, d] bf16 of the owned (token, expert) pairs + their slot map (int32 [n_own * k]:
    destination block row of each pair), computed on the device."""
    d = x.shape[1]
    k = topk_e.shape[1]
    img = torch.empty(ep, C + MR, d, dtype=x.dtype, device=x.device)
    slot = torch.empty(max(1, n_own * k), dtype=torch.int32, device=x.device)
    te = topk_e if topk_e.dtype == torch.int32 else topk_e.to(torch.int32)
    if _gpu(x):
        ext().ep_dispatch(x, te.contiguous(), int(lo), int(n_own), int(El), int(C), img, slot)
    else:
        img.zero_()
        ref.ep_dispatch(x, te, lo, n_own, El, C, img, slot)
    return img, slot


def ep_recv_route(img: torch.Tensor, C: int, El: int) -> "MoERouting":
    """MoERouting over the rows of a received EP image: valid slots sorted stably by local expert."""
    ep = img.shape[0]
    dev = img.device
    if _gpu(img):
        pt = torch.empty(ep * C, dtype=torch.int32, device=dev)
        pw = torch.empty(ep * C, dtype=torch.float32, device=dev)
        eo = torch.empty(El + 1, dtype=torch.int32, device=dev)
        to = torch.empty(El + 1, dtype=torch.int32, device=dev)
        ext().ep_recv_route(img, int(C), int(El), GG_BM, pt, pw, eo, to)
    else:
        pt, pw, eo, to = ref.ep_recv_route(img, C, El, GG_BM)
    rows = img.shape[0] * img.shape[1]  # combine outputs are indexed by image row (topk_* are not read)
    tw = torch.zeros(rows, 1, dtype=torch.float32, device=dev)
    return MoERouting(tw, tw.to(torch.int32), pt, pw, eo, to, El)


def ep_combine(back: torch.Tensor, slot_map: torch.Tensor, topk_w: torch.Tensor, lo: int, n_own: int,
               out: torch.Tensor) -> torch.Tensor:
    """out[i] = sum_j topk_w[lo + i, j] * back_rows[slot_map[i k + j]] for the owned tokens (bf16)."""
    rows = back.reshape(-1, back.shape[-1])
    if n_own <= 0:
        return out
    if _gpu(back):
        ext().ep_combine(rows, slot_map, topk_w.float().contiguous(), int(lo), int(n_own), out)
    else:
        ref.ep_combine(rows, slot_map, topk_w, lo, n_own, out)
    return out
