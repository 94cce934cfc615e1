"""Turns a ScheduledBatch into device tensors, runs the model and samples (one engine step on one GPU/TP rank).

Host->device traffic per step is two packed pinned buffers (one int64: tokens / positions / slots / logit rows;
one int32: block tables / causal limits / decode, cascade and prefill work items) copied with one async H2D each; the only
device->host traffic is the sampled token ids (SURVEY.md §3.2 "device→host: sampled token ids only").

Decode-only batches can be replayed from hipGraphs captured per batch-size bucket (``engine/graphs.py``); mixed
batches run eagerly.
"""
from __future__ import annotations

import bisect

import math
import os
from collections import deque
from dataclasses import dataclass, field

import numpy as np
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.logits_proc import LogitsProcessor, ProcUpdates, spec_forced
from kafka_llm_service_amd.engine.scheduler import ScheduledBatch
from kafka_llm_service_amd.engine.sequence import Sequence
from kafka_llm_service_amd.models.attention import AttnMeta
from kafka_llm_service_amd.models.llama import StepInput, TransformerLM

PAGE = 16
MAX_ITEM_KEYS = 32000  # key range of one attention work item (page ids of an item are staged in 8 KB of LDS)


@dataclass
class HostStep:
    """Host-side plan of one step: packed int64 (tokens | positions | slots | logit rows) and int32 (block tables |
    causal limits | decode items | cascade prefix items | prefill items) buffers plus their layout."""
    B: int = 0
    T: int = 0
    nbt: int = 1
    bt_w: int = 1           # block-table columns (pages of the longest row of the step; a bucket under graphs)
    bt_need: int = 0        # columns holding pages (<= bt_w): what a broadcast plan actually ships
    n_rows: int = 0
    s_total: int = 1        # partial slots per decode row (cascade prefix chunks + suffix pieces)
    n_dec_items: int = 0
    n_prefix_items: int = 0
    cascade_prefix: int = 0  # longest cascade prefix of the step (tokens; 0 = no cascade)
    n_items: int = 0
    prefill_splits: int = 0
    n_merge: int = 0        # prefill row ranges whose tiles were split: i32[-2 n_merge:] = (lo, hi) pairs
    prefix_joined: int = 0  # prefill tiles that ride in the cascade prefix pass (alt partials into prefill_part)
    i64: np.ndarray | None = None
    i32: np.ndarray | None = None
    # (row, seq, position): decode inputs whose token was still being sampled at planning time, filled at launch
    patch: list = field(default_factory=list)
    stats: dict = field(default_factory=dict)
    # rows filled on the device from ModelRunner.tok_buf: i64[late_off : +n_late] = destination token rows,
    # i64[late_off + n_late : +n_late] = source rows of the previous step's sampler output
    n_late: int = 0
    late_off: int = 0


@dataclass
class SampleParams:
    temp: np.ndarray
    topp: np.ndarray
    topk: np.ndarray
    seeds: np.ndarray
    # per-row device logits processing (engine/logits_proc.py): int32 [n, 8] or None when no row needs it
    proc: np.ndarray | None
    greedy: bool
    upd: ProcUpdates | None = None  # table writes (new grammar mask rows, penalty slots to clear) before sampling
    known: dict | None = None       # row -> token fixed by the grammar (forced): the host knows it at launch


_PLAN_SCALARS = ("B", "T", "nbt", "bt_w", "n_rows", "s_total", "n_dec_items", "n_prefix_items", "cascade_prefix",
                 "n_items", "prefill_splits", "n_merge", "n_late", "late_off", "bt_need", "prefix_joined")
PLAN_HDR = 32  # int64 header of a broadcast step plan
PLAN_PAYLOAD_IDX = 1 + len(_PLAN_SCALARS) + 4  # header word holding the payload size (pack_plan)


def pack_plan(h: HostStep, sp: SampleParams) -> tuple[np.ndarray, np.ndarray]:
    """A launched step as (int64 header [PLAN_HDR], uint8 payload): the fixed-layout wire format a TP leader sends its
    followers (two gloo tensor broadcasts per step; no pickling). Everything a follower needs to run the SAME step:
    the layout scalars, the packed int64 / int32 buffers and the sampling parameters with the logits-processing rows
    and table updates (every rank samples the all-gathered logits itself with the same grammar masks and penalty
    counts, so its device copy of the sampled ids — the next step's late decode inputs — is identical to the
    leader's)."""
    n = sp.temp.shape[0]
    i32 = h.i32.astype(np.int32, copy=False)
    nbt_w = h.nbt * h.bt_w
    if 0 < h.bt_need < h.bt_w:  # ship only the block-table columns that hold pages (followers re-pad with zeros)
        bt = i32[:nbt_w].reshape(h.nbt, h.bt_w)[:, :h.bt_need]
        i32 = np.concatenate([bt.reshape(-1), i32[nbt_w:]])
    upd = sp.upd if sp.upd is not None else ProcUpdates()
    proc = sp.proc if sp.proc is not None else np.zeros((0, 8), np.int32)
    parts = [h.i64.astype(np.int64, copy=False), i32,
             sp.temp.astype(np.float32, copy=False), sp.topp.astype(np.float32, copy=False),
             sp.topk.astype(np.int32, copy=False), sp.seeds.astype(np.int64, copy=False),
             proc.astype(np.int32, copy=False), upd.mask_rows.astype(np.int32, copy=False),
             upd.mask_words.astype(np.int32, copy=False), upd.zero_slots.astype(np.int32, copy=False),
             upd.dec.astype(np.int32, copy=False)]
    payload = np.concatenate([np.ascontiguousarray(a).reshape(-1).view(np.uint8) for a in parts])
    hdr = np.zeros(PLAN_HDR, dtype=np.int64)
    hdr[0] = 1
    k = len(_PLAN_SCALARS)
    hdr[1:1 + k] = [getattr(h, f) for f in _PLAN_SCALARS]
    W = upd.mask_words.shape[1] if upd.mask_rows.size else 0
    hdr[1 + k:1 + k + 10] = [h.i64.size, i32.size, n, int(sp.greedy), payload.size, proc.shape[0],
                             upd.mask_rows.size, W, upd.zero_slots.size, upd.dec.shape[0]]
    return hdr, payload


def unpack_plan(hdr: np.ndarray, payload: np.ndarray) -> tuple[HostStep, SampleParams]:
    k = len(_PLAN_SCALARS)
    h = HostStep(**{f: int(v) for f, v in zip(_PLAN_SCALARS, hdr[1:1 + k])})
    n64, n32, n, greedy, _, n_proc, n_mask, W, n_zero, n_dec = (int(v) for v in hdr[1 + k:1 + k + 10])
    o = 0

    def take(dt, cnt):
        nonlocal o
        nb = np.dtype(dt).itemsize * cnt
        a = payload[o:o + nb].view(dt)
        o += nb
        return a

    h.i64 = take(np.int64, n64)
    h.i32 = take(np.int32, n32)
    if 0 < h.bt_need < h.bt_w:  # re-pad the shipped block-table columns to the step's layout width
        nb = h.nbt * h.bt_need
        bt = np.zeros((h.nbt, h.bt_w), dtype=np.int32)
        bt[:, :h.bt_need] = h.i32[:nb].reshape(h.nbt, h.bt_need)
        h.i32 = np.concatenate([bt.reshape(-1), h.i32[nb:]])
    sp = SampleParams(take(np.float32, n), take(np.float32, n), take(np.int32, n), take(np.int64, n), None,
                      bool(greedy))
    proc = take(np.int32, n_proc * 8).reshape(n_proc, 8)
    upd = ProcUpdates(take(np.int32, n_mask), take(np.int32, n_mask * W).reshape(n_mask, W),
                      take(np.int32, n_zero), take(np.int32, 2 * n_dec).reshape(n_dec, 2))
    sp.proc = proc if n_proc else None
    sp.upd = None if upd.empty else upd
    return h, sp


class CollectiveError(RuntimeError):
    """A TP peer stopped taking part in the custom all-reduce (its waits timed out): the step's tokens were computed
    from stale peer data and the replica must fail (503 + respawn), not stream them."""


@dataclass
class Launched:
    tokens: torch.Tensor            # sampled ids (pinned host buffer on GPU, plain tensor on CPU)
    event: object = None            # completion event of the D2H copy
    dev_tokens: torch.Tensor | None = None  # the sampler's device output (input ids of the next step's decode rows)
    rows: dict | None = None        # seq_id -> row of dev_tokens
    err_idx: int | None = None      # slot of ModelRunner._err_host holding the custom all-reduce error word
    known: dict | None = None       # row -> token the grammar forced (known on the host at launch)


MIN_DECODE_KEYS = 256      # smallest key range of one decode work item
# decode workgroups per launch (items x Hkv) the suffix pieces are sized for; 0 = one item per row (no split
# unless a row alone would leave most CUs idle)
# 1,344 with the decode kernel at three workgroups per CU (768 slots): 1,152 was +1.6 % over 768 and 1,344 another
# +0.2-0.4 % over 1,152, same boxes (profiles/r03/decode_occ3/decode_target_ab_*.jsonl; 768 was best at two per CU,
# profiles/r02/decode_items_ab.jsonl)
ROWS_BUCKETS = (64, 96, 128, 256, 1 << 30)  # step-size histogram buckets (decode GEMM row-tile plans, skinny, BLAS)
DECODE_TARGET_ITEMS = 1344  # (768 / 1536 / 2304 lose to it: profiles/r04/bench_ab_decode_target_blas.jsonl)
MAX_PARTIALS = 64           # partial slots per row that the decode kernel's fused merge reads (one lane each)
MAX_PREFIX_CHUNKS = 32


def pad_step_rows(T: int) -> int:
    """Token rows of a mixed step whose GEMMs go to hipBLASLt (129..256 rows): measured on MI355X (Llama-3-8B shapes,
    ``benchmarks/gemm_bench.py``, profiles/r02/gemm_sweep_M129_320.log) the library picks slow kernels for 129..152
    rows (QKV 40 vs 26 us) and at multiples of 32 (down-proj at 192 rows: 101 vs 60 us), so the step is padded with
    inert rows (no KV slot, no attention item, no logits) to the next 16 k + 8 >= 168."""
    if T <= ops.STREAM_MAX_M or T > 256:  # (steps the streaming GEMM takes need no padding)
        return T
    t = max(T, 168)
    t += (8 - t % 16) % 16
    return t if t <= 256 else T


def plan_prefill_items(tiles: list[tuple], hkv: int, target_wgs: int, min_chunk: int,
                       max_keys: int = MAX_ITEM_KEYS) -> tuple[list[tuple], int, list[tuple[int, int]]]:
    """Work items of the prefill tile kernel from query tiles (q0, count, bt_row, extent, hi[, lo, s0]): ``extent`` =
    keys the tile attends (its last token's position + 1), ``hi`` = key bound of the chunk. A tile with ``lo`` > 0
    attends only keys [lo, extent) — its keys below lo (a shared system prefix) were attended by the step's cascade
    prefix pass, whose partials sit in slots [0, s0) of the row — so it always writes partials, at slots s0, s0 + 1, ...

    The tile kernel's time per workgroup is ~a + b x (32-key blocks), so a launch is as long as its longest item. A
    causal prompt's tiles grow linearly (a 2k prompt: 2 .. 64 blocks) and a new turn's few tiles each span a ~20k-token
    context: when the launch is at most ~two rounds of workgroups, tiles longer than the balanced share
    (sum of extents x Hkv / target_wgs, >= min_chunk) are split into equal key pieces whose (O, lse) partials are
    merged afterwards; shorter tiles still write bf16 rows directly. Larger launches only get longest-first order
    (the dispatcher then packs the tail). Returns (items, partial slots per row, merged row ranges)."""
    if not tiles:
        return [], 0, []
    tiles = [tuple(t) + (0, 0) if len(t) == 5 else tuple(t) for t in tiles]
    total = sum(t[3] - t[5] for t in tiles) * hkv
    longest = max(t[3] - t[5] for t in tiles)
    if len(tiles) * hkv >= 2 * target_wgs:
        ck = max_keys  # many tiles: split only what exceeds the LDS page-staging bound
    else:
        ck = min(max(min_chunk, -(-total // (target_wgs * 32)) * 32), max_keys)
        if longest < 3 * ck // 2 and longest <= max_keys:
            ck = max_keys  # nothing long enough for a split to shorten the launch by much
        elif all(t[3] - t[5] > ck for t in tiles):
            # every tile is split (new turns against a long cached context): keep the launch to ONE round of
            # workgroups — per-tile rounding up can overshoot target_wgs by a few, and a second round of a handful
            # of workgroups doubles the launch (r03 trace: 272 workgroups for a new turn, 125 us vs ~60)
            while ck < max_keys and sum(-(-(t[3] - t[5]) // ck) for t in tiles) * hkv > target_wgs:
                ck += 32
    items, splits, ranges = [], 0, []
    for q0, cnt, btr, ext, hi, lo, s0 in tiles:
        span = ext - lo
        if span <= ck and lo == 0:
            items.append((q0, cnt, btr, 0, hi, -1, 0, 0))
            continue
        nsp = max(1, -(-span // ck))
        ps = -(-span // (nsp * 32)) * 32
        nsp = -(-span // ps)
        items += [(q0, cnt, btr, lo + c * ps, min(hi, lo + (c + 1) * ps), s0 + c, 0, 0) for c in range(nsp)]
        splits = max(splits, s0 + nsp)
        if ranges and ranges[-1][1] == q0:
            ranges[-1] = (ranges[-1][0], q0 + cnt)
        else:
            ranges.append((q0, q0 + cnt))
    items.sort(key=lambda it: it[3] - it[4])  # longest key range first
    return items, splits, ranges


def retile(spans: list[tuple[int, int]], tile: int) -> list[tuple[int, int]]:
    """(q0, count) token spans (ascending) -> the same tokens as (q0, count) tiles of at most ``tile`` tokens, contiguous
    spans joined first: 8 new turns of 30 tokens back to back make 4 full tiles, not 8 half-empty ones."""
    if tile <= 0:  # (off: the spans as they are)
        return [tuple(t) for t in spans]
    runs: list[list[int]] = []
    for q0, cnt in spans:
        if runs and runs[-1][0] + runs[-1][1] == q0:
            runs[-1][1] += cnt
        else:
            runs.append([q0, cnt])
    return [(q0 + t, min(tile, cnt - t)) for q0, cnt in runs for t in range(0, cnt, tile)]


def merge_ranges(ranges: list[tuple[int, int]]) -> list[tuple[int, int]]:
    """Sorted union of half-open row ranges, touching ones joined (one attn_merge launch per range)."""
    out: list[tuple[int, int]] = []
    for lo, hi in sorted(ranges):
        if out and lo <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], hi))
        else:
            out.append((lo, hi))
    return out


def prefix_groups(bt: np.ndarray, nfull: np.ndarray, min_blocks: int) -> tuple[list[int], list[tuple[int, int]]]:
    """Cascade groups of decode rows: rows whose block tables start with the same pages share that KV prefix.

    ``bt`` int32 [B, W] block tables, ``nfull[b]`` = pages of row b that may belong to a shared prefix (full pages
    before the one holding the current token). Returns (order, groups): a permutation of the rows that makes every
    group contiguous, and (row_count, prefix_pages) per group in that order (groups first, then ungrouped rows).
    A set of rows is split by the first page where it disagrees when its common prefix is shorter than
    ``min_blocks`` — e.g. threads on the Kafka system prompt vs threads created with their own system message
    (quirk Q4 of SURVEY.md §2.9) vs stateless /chat/completions traffic each get their own group."""
    groups: list[tuple[list[int], int]] = []
    loose: list[int] = []

    def rec(rows: np.ndarray, d: int) -> None:
        while True:
            if len(rows) < 2:
                loose.extend(rows.tolist())
                return
            lim = int(nfull[rows].min())
            sub = bt[rows, d:lim]
            if sub.shape[1]:
                eq = (sub == sub[0]).all(0)
                j = d + (int(np.argmin(eq)) if not eq.all() else sub.shape[1])
            else:
                j = d
            if j >= min_blocks:
                groups.append((rows.tolist(), j))
                return
            short = nfull[rows] <= j  # rows without a page j: cannot share anything longer
            if short.any():
                loose.extend(rows[short].tolist())
                rows = rows[~short]
                d = j
                continue
            col = bt[rows, j]
            for v in np.unique(col):
                rec(rows[col == v], j + 1)
            return

    rec(np.arange(bt.shape[0]), 0)
    order = [r for rows, _ in groups for r in rows] + loose
    return order, [(len(rows), p) for rows, p in groups]


def decode_items(seq_lens: np.ndarray, kv_start: np.ndarray, npre: np.ndarray, hkv: int,
                 target: int = DECODE_TARGET_ITEMS, min_keys: int = MIN_DECODE_KEYS) -> np.ndarray:
    """Work items (b, lo, hi, split, nsplit, npre, 0, 0) of the decode kernel: every row's keys [kv_start, len) in
    32-key-aligned pieces of about ``ch`` keys, ``ch`` chosen so the launch has ~``target`` workgroups (x Hkv) of
    about equal bytes (long histories are split, short ones stay whole); at most MAX_PARTIALS - npre pieces."""
    B = seq_lens.shape[0]
    suffix = np.maximum(seq_lens - kv_start, 1).astype(np.int64)
    # fewer rows than it takes to fill the GPU (B x Hkv < 512 workgroups): split so the launch still has ~512
    target = max(target, 512) if B * hkv < 512 else target
    if target <= 0:
        ch = int(suffix.max())
    else:
        ch = max(min_keys, -(-int(suffix.sum()) * hkv // (target * 32)) * 32)
    a0 = kv_start - kv_start % 32
    nb = (seq_lens - a0 + 31) // 32
    ns = np.minimum(np.maximum(1, -(-suffix // ch)), MAX_PARTIALS - npre)
    bps = -(-nb // ns)
    ns = -(-nb // bps)  # no empty trailing piece
    rows = np.repeat(np.arange(B), ns)
    first = np.cumsum(ns) - ns
    split = np.arange(rows.shape[0]) - np.repeat(first, ns)
    lo = np.maximum(kv_start[rows], a0[rows] + split * bps[rows] * 32)
    hi = np.minimum(seq_lens[rows], a0[rows] + (split + 1) * bps[rows] * 32)
    z = np.zeros_like(rows)
    it = np.stack([rows, lo, hi, split, ns[rows], npre[rows], z, z], 1).astype(np.int32)
    if ns.max() > 1:  # longest pieces first: they start while the dispatcher fills the GPU, short ones fill the tail
        it = it[np.argsort(it[:, 1] - it[:, 2], kind="stable")]
    return it


def decode_items_fixed(seq_lens: np.ndarray, kv_start: np.ndarray, npre: np.ndarray, hkv: int,
                       target: int = DECODE_TARGET_ITEMS) -> np.ndarray:
    """``decode_items`` with EXACTLY n = max(B, target // hkv) items (a captured decode graph's launch shape then
    depends on B alone, no padded grid): the n pieces are dealt to the rows in proportion to their 32-key blocks
    (largest remainder, at least one per row, at most MAX_PARTIALS - npre and one per block), each row's blocks split
    evenly; rows too short to take their share leave null items (split -1: the kernel drops them)."""
    B = seq_lens.shape[0]
    n = max(B, target // hkv)
    a0 = kv_start - kv_start % 32
    nb = np.maximum((seq_lens - a0 + 31) // 32, 1).astype(np.int64)
    cap = np.maximum(1, np.minimum(nb, MAX_PARTIALS - npre))
    ns = np.minimum(cap, np.maximum(1, (n * nb) // max(1, int(nb.sum()))))
    while int(ns.sum()) > n:  # the at-least-one floor overshot: take pieces back from the lightest split rows
        more = ns > 1
        if not more.any():
            break
        load = np.where(more, nb / ns, np.inf)
        ns[int(np.argmin(load))] -= 1
    left = n - int(ns.sum())
    while left > 0:  # largest blocks-per-piece first
        room = ns < cap
        if not room.any():
            break
        load = np.where(room, nb / ns, -1.0)
        k = min(left, int(room.sum()))
        for b in np.argsort(-load, kind="stable")[:k]:
            ns[b] += 1
        left = n - int(ns.sum())
    rows = np.repeat(np.arange(B), ns)
    first = np.cumsum(ns) - ns
    split = np.arange(rows.shape[0]) - np.repeat(first, ns)
    b_lo = (split * nb[rows]) // ns[rows]
    b_hi = ((split + 1) * nb[rows]) // ns[rows]
    lo = np.maximum(kv_start[rows], a0[rows] + b_lo * 32)
    hi = np.minimum(seq_lens[rows], a0[rows] + b_hi * 32)
    z = np.zeros_like(rows)
    it = np.stack([rows, lo, hi, split, ns[rows], npre[rows], z, z], 1).astype(np.int32)
    it = it[np.argsort(it[:, 1] - it[:, 2], kind="stable")]
    if it.shape[0] < n:
        pad = np.zeros((n - it.shape[0], 8), dtype=np.int32)
        pad[:, 3] = -1
        it = np.concatenate([it, pad])
    return it


_NP2TORCH = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32}


class _Stager:
    """Per-step host->device uploads through a ring of pinned staging arenas (one arena per launch, bump-allocated):
    no pinned allocation and no pageable copy on the step path, so every upload is a plain async DMA in stream
    order. An arena is reused ``depth`` launches later, when at most two steps can be in flight — its copies have
    executed by then."""

    def __init__(self, device: torch.device, nbytes: int = 8 << 20, depth: int = 4):
        self.device = device
        self.nbytes = nbytes
        self.bufs: list[torch.Tensor | None] = [None] * depth
        self.events: list = [None] * depth  # copies of the arena's last launch (a TP follower is not throttled)
        self.i = 0
        self.off = 0

    def begin(self) -> None:
        if self.device.type == "cuda":
            ev = self.events[self.i]
            if ev is None:
                ev = self.events[self.i] = torch.cuda.Event()
            ev.record()  # after every copy issued from the arena that is being left
        self.i = (self.i + 1) % len(self.bufs)
        self.off = 0
        ev = self.events[self.i]
        if ev is not None:
            ev.synchronize()  # normally long done: the arena's copies ran len(bufs) launches ago

    def upload_many(self, arrays: list[np.ndarray]) -> list[torch.Tensor]:
        """Several arrays staged back to back (256-B aligned) and moved by ONE async copy into one device buffer —
        a step's plan and sampling parameters cost one copy launch instead of one each; returns device views."""
        arrays = [np.ascontiguousarray(a) for a in arrays]
        if self.device.type != "cuda":
            return [torch.from_numpy(a) for a in arrays]
        offs, off = [], 0
        for a in arrays:
            offs.append(off)
            off = (off + a.nbytes + 255) & ~255
        base = (self.off + 255) & ~255
        buf = self.bufs[self.i]
        if buf is None or base + off > buf.numel():
            self.bufs[self.i] = buf = torch.empty(max(self.nbytes, 2 * (base + off)), dtype=torch.uint8,
                                                  pin_memory=True)
        host = buf.numpy()
        for a, o in zip(arrays, offs):
            host[base + o:base + o + a.nbytes] = a.reshape(-1).view(np.uint8)
        self.off = base + off
        dev = torch.empty(off, dtype=torch.uint8, device=self.device)
        dev.copy_(buf[base:base + off], non_blocking=True)
        return [dev[o:o + a.nbytes].view(_NP2TORCH[a.dtype]).view(a.shape) for a, o in zip(arrays, offs)]

    def upload(self, a: np.ndarray) -> torch.Tensor:
        a = np.ascontiguousarray(a)
        if self.device.type != "cuda":
            return torch.from_numpy(a)
        nb = a.nbytes
        off = (self.off + 255) & ~255
        buf = self.bufs[self.i]
        if buf is None or off + nb > buf.numel():
            # (a replaced arena goes back to torch's pinned cache, which waits for its recorded copies)
            self.bufs[self.i] = buf = torch.empty(max(self.nbytes, 2 * (off + nb)), dtype=torch.uint8,
                                                  pin_memory=True)
        stage = buf[off:off + nb]
        stage.numpy()[:] = a.reshape(-1).view(np.uint8)
        self.off = off + nb
        dev = torch.empty(a.size, dtype=_NP2TORCH[a.dtype], device=self.device)
        dev.view(torch.uint8).copy_(stage, non_blocking=True)
        return dev.view(a.shape)

    def upload_into(self, arrays: list[np.ndarray | None], offs: list[int], dst: torch.Tensor) -> None:
        """Arrays staged at their byte offsets of ``dst`` (a uint8 device buffer whose layout the caller fixed) and moved
        by ONE async copy of the whole range — a hipGraph's static inputs refreshed with one copy launch instead of an
        upload plus a device copy per array. Every byte of ``dst`` is written: the ranges of None arrays (and any
        padding) become zeros, never stale bytes of an earlier upload."""
        n = dst.numel()
        if self.device.type != "cuda":
            dst.zero_()
            for a, o in zip(arrays, offs):
                if a is not None:
                    dst[o:o + a.nbytes].copy_(torch.from_numpy(np.ascontiguousarray(a).reshape(-1).view(np.uint8)))
            return
        base = (self.off + 255) & ~255
        buf = self.bufs[self.i]
        if buf is None or base + n > buf.numel():
            self.bufs[self.i] = buf = torch.empty(max(self.nbytes, 2 * (base + n)), dtype=torch.uint8, pin_memory=True)
        host = buf.numpy()
        host[base:base + n] = 0
        for a, o in zip(arrays, offs):
            if a is not None:
                a = np.ascontiguousarray(a)
                host[base + o:base + o + a.nbytes] = a.reshape(-1).view(np.uint8)
        self.off = base + n
        dst.copy_(buf[base:base + n], non_blocking=True)


class ModelRunner:
    def __init__(self, model: TransformerLM, k_caches, v_caches, kvm, max_num_seqs: int, max_blocks_per_seq: int,
                 cascade_min_prefix: int = 512, use_cascade: bool = True, target_wgs: int = 256,
                 prefill_kv_chunk: int = 1024):
        self.model = model
        self.k_caches, self.v_caches = k_caches, v_caches
        self.kvm = kvm
        self.device = model.device
        self.max_num_seqs = max_num_seqs
        self.max_blocks = max_blocks_per_seq
        self.G = model.hq // model.hkv
        # tile-kernel variant (ops.tile_rows): 3 = LDS-DMA ring kernel (csrc/attn_tile.hip, 8 waves x 256 query rows,
        # bf16 pages); 0 = register-staged 8 waves x 256 rows (fp8 pages); 1 = 4 waves x 128 rows
        fp8 = bool(k_caches) and ops.is_fp8_cache(k_caches[0])
        self.variant = int(os.environ.get("KAFKA_TILE_VARIANT", "0" if fp8 else "3"))
        if fp8 and self.variant == 3:
            raise ValueError("tile variant 3 reads bf16 KV pages only")
        # mixed steps of 129..256 rows padded away from hipBLASLt's slow sizes (dense TP = 1 GPU models)
        self.pad_rows = (self.device.type == "cuda" and model.tp == 1 and not getattr(model, "tiled_only", False)
                         and os.environ.get("KAFKA_PAD_ROWS", "1") == "1")
        self.tile = ops.tile_rows(self.variant) // self.G  # tokens per attention work item
        # the v3 cascade hands its prefix partials to the decode kernel as bf16 (normalised O, fp32 lse): ~33 MB
        # less HBM traffic per Llama-3-8B layer at 64 threads on an 18k prefix (+1.4 %,
        # profiles/r03/bench_ab_cascade_bf16_partials.jsonl)
        self.cascade_bf16 = self.variant == 3
        self.cascade_min_prefix = cascade_min_prefix
        self.target_wgs = target_wgs  # workgroups the prefill / cascade tile launches are balanced for
        self.prefill_kv_chunk = int(os.environ.get("KAFKA_PREFILL_KV_CHUNK", prefill_kv_chunk))
        self.use_cascade = use_cascade
        self.vocab = model.cfg.vocab_size
        pin = self.device.type == "cuda"
        self._pin = pin
        self.last_stats: dict = {}
        self.recent_stats: deque = deque(maxlen=16)  # stats of the last launched steps (two can be in flight)
        self.rows_hist = [0] * len(ROWS_BUCKETS)  # launched steps by token rows (ROWS_BUCKETS upper bounds)
        self.broadcast = None  # set on a TP leader: callable(HostStep, SampleParams) (engine/tp_worker.py)
        self._tok_host = None  # pinned landing buffers of the sampled ids
        self._err_host = None  # pinned landing slots of the custom all-reduce error word (TP)
        self.stager = _Stager(self.device)
        # every step's sampled ids also land here (fixed address, so hipGraphs can read it): the next step's decode
        # rows whose token was still being sampled at launch gather their input ids from it on the stream
        self.tok_buf = torch.zeros(max_num_seqs * 2 + 64, dtype=torch.int64, device=self.device)
        self.graphs = None  # engine/graphs.py DecodeGraphs when hipGraph decode is enabled
        # decode_items_fixed without graphs too (equivalence tests; KAFKA_FIXED_DECODE_ITEMS=1 separates the graph
        # plan's cost from the replay's in an eager A/B)
        self.fixed_decode_items = os.environ.get("KAFKA_FIXED_DECODE_ITEMS", "0") == "1"
        # a joined new turn's own keys (its history behind the shared prefix) ride in the cascade launch too
        self.join_suffix = os.environ.get("KAFKA_JOIN_SUFFIX", "1") == "1"
        self.retile_joins = os.environ.get("KAFKA_RETILE_JOINS", "1") == "1"  # (model_runner.retile)
        self.step_events: list | None = None  # (start, end) timing events per launched step when a list is set
        # grammar masks / forced tokens / penalties inside the sampler kernel (tables allocated on first use)
        self.lp = LogitsProcessor(self.device, self.vocab, max_slots=max(256, max_num_seqs))

    # ------------------------------------------------------------------------------------------------------------
    def prepare(self, batch: ScheduledBatch) -> tuple[StepInput, list[Sequence]]:
        host, sample_seqs = self.build_host(batch)
        return self.to_device(host), sample_seqs

    def build_host(self, batch: ScheduledBatch) -> tuple[HostStep, list[Sequence]]:
        """All host-side work of a step: token/slot/page-table packing and attention work-item planning. The result
        is a few numpy arrays + scalars — what a TP leader broadcasts to its followers (``engine/tp_worker.py``).

        Decode rows are reordered so that every cascade group (rows sharing a KV prefix of at least
        ``cascade_min_prefix`` tokens, ``prefix_groups``) is contiguous: each group's prefix is attended once for all
        its rows by the tile kernel, the per-row suffixes by the decode kernel in pieces of about equal size."""
        dec = list(batch.decode)
        B = len(dec)
        pre = batch.prefill
        T_real = B + sum(e - s for _, s, e in pre)
        T = pad_step_rows(T_real) if self.pad_rows else T_real
        rows = B + len(pre)
        nbt = max(1, rows)
        need = max([-(-s.total_len // PAGE) for s in dec] + [-(-b // PAGE) for _, _, b in pre] + [1])
        # under graphs the width is a power-of-two bucket (>= 64 pages): the layout (and so the captured graph)
        # changes only when the longest row crosses a bucket, and the per-step upload / TP broadcast stays small
        bt_w = (min(self.max_blocks, max(64, 1 << (need - 1).bit_length())) if self.graphs is not None
                else min(self.max_blocks, -(-need // 16) * 16))
        bt = np.zeros((nbt, bt_w), dtype=np.int32)
        groups: list[tuple[int, int]] = []
        seq_lens = np.fromiter((s.total_len for s in dec), dtype=np.int64, count=B)
        if B:
            self.kvm.fill_block_tables([s.seq_id for s in dec], bt)
            if self.use_cascade and B >= 2:
                nfull = (seq_lens - 1) // PAGE
                order, groups = prefix_groups(bt[:B], nfull, -(-self.cascade_min_prefix // PAGE))
                if groups and order != list(range(B)):
                    dec = [dec[i] for i in order]
                    bt[:B] = bt[:B][order]
                    seq_lens = seq_lens[order]
        if pre:
            self.kvm.fill_block_tables([s.seq_id for s, _, _ in pre], bt[B:])
        # ---- int64 pack: tokens | positions | slots | logit_rows
        tokens = np.empty(T, dtype=np.int64)
        positions = np.empty(T, dtype=np.int64)
        slots = np.empty(T, dtype=np.int64)
        q_limit = np.empty(T, dtype=np.int32)
        sample_seqs: list[Sequence] = []
        logit_rows: list[int] = []
        patch = []
        for i, s in enumerate(dec):
            p = s.total_len - 1
            t = s.token_at(p)
            if t < 0:  # PENDING: sampled by the step still in flight (async scheduling)
                patch.append((i, s, p))
            tokens[i] = t
            positions[i] = p
            q_limit[i] = p
            self.kvm.fill_slots(s.seq_id, p, p + 1, slots, i)
            sample_seqs.append(s)
            logit_rows.append(i)
        tiles = []
        r = B
        for j, (s, a, b) in enumerate(pre):
            n = b - a
            tokens[r:r + n] = s.tokens_range(a, b)
            positions[r:r + n] = np.arange(a, b)
            q_limit[r:r + n] = np.arange(a, b, dtype=np.int32)
            self.kvm.fill_slots(s.seq_id, a, b, slots, r)
            bt_row = B + j
            for t0 in range(0, n, self.tile):
                cnt = min(self.tile, n - t0)
                tiles.append((r + t0 - B, cnt, bt_row, a + t0 + cnt, b))
            if b == s.total_len:
                sample_seqs.append(s)
                logit_rows.append(r + n - 1)
            r += n
        if T > T_real:  # inert padding rows: token 0 at position 0, no KV write, not attended, no logits
            tokens[T_real:] = 0
            positions[T_real:] = 0
            slots[T_real:] = -1
            q_limit[T_real:] = 0
        # ---- decode metadata (+ cascade over each group's shared prefix)
        h = HostStep(B=B, T=T, nbt=nbt, bt_w=bt_w, bt_need=min(need, bt_w), n_rows=len(logit_rows), patch=patch)
        i32_parts = [bt.reshape(-1), q_limit]
        # new-turn prefill chunks whose block table starts with a cascade group's prefix pages (the ~18k shared
        # system prompt every new turn of a thread re-attends): their tokens join the group's prefix pass — one read
        # of the prefix pages per step for all rows — and their own tiles attend only the keys behind the prefix
        joins = self._prefix_joins(bt, B, pre, groups, tiles) if groups and self.variant == 3 else {}
        sfx_slots, sfx_rows = 0, []  # joined tiles whose own keys are planned into the prefix pass: slots, rows
        if B:
            kv_start = np.zeros(B, dtype=np.int64)
            npre = np.zeros(B, dtype=np.int64)
            pit = []
            if groups:
                # joined tiles' own key spans (behind the prefix): with join_suffix they are items of this launch too
                spans = {ti: tiles[ti][3] - groups[gi][1] * PAGE for gi, js in joins.items() for ti in js} \
                    if self.join_suffix else {}
                # the joined rows' prefix-pass tiles: the group's joined tokens re-tiled at token granularity (a burst
                # of short new turns fills 64-token tiles instead of one mostly empty tile per turn; every key of the
                # prefix is below every joined token's position, so tokens of different turns share a tile)
                jt = {gi: retile([tiles[ti][:2] for ti in js], self.tile if self.retile_joins else 0)
                      for gi, js in joins.items()}
                # key chunks sized so the prefix pass launches ~target_wgs workgroups over all groups together
                work = sum(-(-n // self.tile) * p * PAGE for n, p in groups) + \
                    sum(len(t) * groups[gi][1] * PAGE for gi, t in jt.items()) + sum(spans.values())
                want = max(1, self.target_wgs // self.model.hkv)
                chunk = min(MAX_ITEM_KEYS, max(256, -(-work // (want * 32)) * 32))
                # one round of workgroups: per-group rounding up can overshoot the target by a few items, and a
                # second round of a handful of workgroups doubles the launch
                tiles_per_group = [-(-n // self.tile) + len(jt.get(gi, ())) for gi, (n, _) in enumerate(groups)]
                while chunk < MAX_ITEM_KEYS and sum(t * -(-(p * PAGE) // chunk) for t, (_, p) in
                                                    zip(tiles_per_group, groups)) + \
                        sum(-(-sp // chunk) for sp in spans.values()) > want:
                    chunk += 32
                r0 = 0
                for gi, (n, p) in enumerate(groups):
                    P = p * PAGE
                    nc = -(-P // chunk)
                    ck = chunk
                    if nc > MAX_PREFIX_CHUNKS:
                        ck = -(-P // (MAX_PREFIX_CHUNKS * 32)) * 32
                        nc = -(-P // ck)
                    for c in range(nc):  # chunk-major: the row tiles of one chunk run together (L2 sharing)
                        for g0 in range(r0, r0 + n, self.tile):
                            pit.append((g0, min(self.tile, r0 + n - g0), r0, c * ck, min(P, (c + 1) * ck), c, 0, 0))
                        for q0, cnt in jt.get(gi, ()):  # joined prefill rows: q rows B + q0, fp32 alt partials
                            pit.append((B + q0, cnt, r0, c * ck, min(P, (c + 1) * ck), c, 1, 0))
                    for ti in joins.get(gi, ()):
                        tiles[ti] = tiles[ti][:5] + (P, nc)
                        if ti in spans:
                            # the tile's keys [P, extent) in pieces of ~chunk keys: alt partials at slots nc, nc + 1..
                            # (beside its prefix pieces' slots 0..nc-1), so the step needs no separate prefill launch
                            # for it; attn_merge combines all of the row's slots as before
                            q0, cnt, btr, ext, hi = tiles[ti][:5]
                            nsp = max(1, -(-spans[ti] // chunk))
                            ps = -(-spans[ti] // (nsp * 32)) * 32
                            nsp = -(-spans[ti] // ps)
                            pit += [(B + q0, cnt, btr, P + c * ps, min(hi, P + (c + 1) * ps), nc + c, 1, 0)
                                    for c in range(nsp)]
                            sfx_slots = max(sfx_slots, nc + nsp)
                            sfx_rows.append((q0, q0 + cnt))
                    kv_start[r0:r0 + n] = P
                    npre[r0:r0 + n] = nc
                    h.cascade_prefix = max(h.cascade_prefix, P)
                    r0 += n
            self._plan_decode_items(h, seq_lens, kv_start, npre, i32_parts)
            if pit:
                h.n_prefix_items = len(pit)
                i32_parts.append(np.asarray(pit, dtype=np.int32).reshape(-1))
        if sfx_rows:  # (their suffix items are in the prefix pass)
            done = {ti for js in joins.values() for ti in js}
            tiles = [t for ti, t in enumerate(tiles) if ti not in done]
        if tiles or sfx_rows:
            # long tiles (a new turn against a ~20k-token cached context, the late tiles of a causal prompt) are
            # split along the key range so the launch is balanced; their partials are merged afterwards
            items, h.prefill_splits, ranges = plan_prefill_items(tiles, self.model.hkv, self.target_wgs,
                                                                 min(256, self.prefill_kv_chunk))
            if sfx_rows:
                h.prefill_splits = max(h.prefill_splits, sfx_slots)
                ranges = merge_ranges(ranges + sfx_rows)
            h.n_items = len(items)
            i32_parts.append(np.asarray(items, dtype=np.int32).reshape(-1))
            if ranges:
                h.n_merge = len(ranges)
                i32_parts.append(np.asarray(ranges, dtype=np.int32).reshape(-1))
        h.i64 = np.concatenate([tokens, positions, slots, np.asarray(logit_rows, dtype=np.int64)])
        h.i32 = np.concatenate(i32_parts)
        h.prefix_joined = sum(len(v) for v in joins.values())
        h.stats = {"B": B, "T": T, "cascade_prefix": h.cascade_prefix, "cascade_groups": len(groups),
                   "prefix_joined_tiles": h.prefix_joined,
                   "decode_items": h.n_dec_items, "prefix_items": h.n_prefix_items, "s_total": h.s_total,
                   "prefill_splits": h.prefill_splits, "prefill_items": h.n_items}
        return h, sample_seqs

    @staticmethod
    def _prefix_joins(bt: np.ndarray, B: int, pre: list, groups: list[tuple[int, int]],
                      tiles: list[tuple]) -> dict[int, list[int]]:
        """{group index: prefill tile indices} of the prefill chunks that start at or behind a cascade group's
        shared prefix and whose block table holds the same prefix pages (the groups' rows are contiguous from row
        0 in group order; a tile names its chunk through its block-table row B + j)."""
        starts, r0 = [], 0
        for n, p in groups:
            starts.append((r0, p))
            r0 += n
        chunk_group: dict[int, int] = {}
        for j, (s, a, b) in enumerate(pre):
            for gi, (g_row, p) in enumerate(starts):
                if a >= p * PAGE and np.array_equal(bt[B + j, :p], bt[g_row, :p]):
                    chunk_group[B + j] = gi
                    break
        joins: dict[int, list[int]] = {}
        for ti, t in enumerate(tiles):
            gi = chunk_group.get(t[2])
            if gi is not None:
                joins.setdefault(gi, []).append(ti)
        return joins

    def _plan_decode_items(self, h: HostStep, seq_lens: np.ndarray, kv_start: np.ndarray, npre: np.ndarray,
                           i32_parts: list) -> None:
        if self.graphs is not None or self.fixed_decode_items:  # graph replay: the decode grid depends on B alone
            ditems = decode_items_fixed(seq_lens, kv_start, npre, self.model.hkv)
        else:
            ditems = decode_items(seq_lens, kv_start, npre, self.model.hkv)
        h.n_dec_items = int(ditems.shape[0])
        real = ditems[:, 3] >= 0
        h.s_total = int((npre[ditems[real, 0]] + ditems[real, 4]).max()) if h.B else 1
        if self.graphs is not None:
            # (a graph layout key: rounded up to a multiple of 8 so a handful of layouts cover every step; the
            # partial buffers' unused slots are never touched)
            h.s_total = min(MAX_PARTIALS, -(-h.s_total // 8) * 8)
        i32_parts.append(ditems.reshape(-1))

    def to_device(self, h: HostStep, sp: "SampleParams | None" = None) -> StepInput:
        """One H2D copy of the packed buffers (and of the step's sampling parameters when ``sp`` samples with
        temperature: left in ``self._sp_dev`` for ``sample_device``), then views into it (identical on every TP
        rank)."""
        arrays = [h.i64, h.i32]
        if sp is not None and not sp.greedy and sp.temp.shape[0]:
            arrays += [np.concatenate([sp.temp, sp.topp]), sp.topk, sp.seeds]
        if sp is not None and sp.proc is not None:
            arrays.append(sp.proc)
        dev = self.stager.upload_many(arrays)
        if len(dev) > 2:
            has_t = not sp.greedy and sp.temp.shape[0]
            self._sp_dev = (sp, *(dev[2:5] if has_t else (None, None, None)), dev[-1] if sp.proc is not None else None)
        return self.views(dev[0], dev[1], h)

    def views(self, d64: torch.Tensor, d32: torch.Tensor, h: HostStep) -> StepInput:
        """StepInput over packed device buffers laid out as ``h`` describes (only h's scalars are read, so a hipGraph
        captured over static buffers replays with any step of the same layout)."""
        B, T, nbt = h.B, h.T, h.nbt
        t_tokens, t_pos, t_slots = d64[0:T], d64[T:2 * T], d64[2 * T:3 * T]
        t_rows = d64[3 * T:3 * T + h.n_rows]
        meta = AttnMeta(num_decode=B, num_tokens=T, scale=self.model.scale, variant=self.variant)
        o = 0
        n_bt = nbt * h.bt_w
        meta.block_tables = d32[o:o + n_bt].view(nbt, h.bt_w)
        o += n_bt
        meta.q_limit = d32[o:o + T]
        o += T
        Hq, D = self.model.hq, self.model.D
        if B:
            meta.decode_items = d32[o:o + h.n_dec_items * 8].view(-1, 8)
            o += h.n_dec_items * 8
            if h.n_prefix_items:
                meta.prefix_items = d32[o:o + h.n_prefix_items * 8].view(-1, 8)
                o += h.n_prefix_items * 8
            meta.s_total = h.s_total
            meta.part = torch.empty(B, Hq, h.s_total, D, dtype=torch.float32, device=self.device)
            meta.lse = torch.empty(B, Hq, h.s_total, dtype=torch.float32, device=self.device)
            if h.n_prefix_items and self.cascade_bf16:
                meta.pre_part = torch.empty(B, Hq, h.s_total, D, dtype=torch.bfloat16, device=self.device)
            meta.extra["cascade_prefix"] = h.cascade_prefix
        if h.n_items or h.n_merge:
            if h.n_items:
                meta.prefill_items = d32[o:o + h.n_items * 8].view(-1, 8)
                o += h.n_items * 8
            if h.prefill_splits:
                Tp = T - B
                meta.prefill_splits = h.prefill_splits
                mr = h.i32[h.i32.size - 2 * h.n_merge:].reshape(-1, 2)  # host copy of the plan (every TP rank)
                meta.prefill_merge = [(int(lo), int(hi)) for lo, hi in mr]
                meta.prefill_part = torch.empty(Tp, Hq, h.prefill_splits, D, dtype=torch.float32,
                                                device=self.device)
                meta.prefill_lse = torch.full((Tp, Hq, h.prefill_splits), float("-inf"), dtype=torch.float32,
                                              device=self.device)
                meta.prefix_joined = h.prefix_joined > 0
        if h.n_late:
            L, n = h.late_off, h.n_late
            t_tokens.index_copy_(0, d64[L:L + n], self.tok_buf.index_select(0, d64[L + n:L + 2 * n]))
        return StepInput(t_tokens, t_pos, t_slots, meta, t_rows)

    def _host(self, a: np.ndarray) -> torch.Tensor:
        """Host tensor of ``a`` for an async copy into a device buffer (pinned on GPU hosts)."""
        t = torch.from_numpy(a)
        return t.pin_memory() if self.device.type == "cuda" else t

    def _h2d(self, a: np.ndarray) -> torch.Tensor:
        return self.stager.upload(a)

    # ------------------------------------------------------------------------------------------------------------
    def sample(self, logits: torch.Tensor, seqs: list[Sequence]) -> torch.Tensor:
        return self.sample_device(logits, self.sample_params(seqs))

    def sample_params(self, seqs: list[Sequence]) -> "SampleParams":
        """Per-row sampling parameters of a step; rows with a token constraint or penalties get a logits-processing
        row (engine/logits_proc.py) that the sampler kernel applies on the device. A constrained row's spec is
        computed from its landed tokens, or past a pending one when the grammar can guess its successor state
        (engine/constrained.py: a wrong guess rolls the row back one token); a forced token is returned in
        ``known`` so the engine writes it at launch."""
        n = len(seqs)
        temp = np.empty(n, dtype=np.float32)
        topp = np.empty(n, dtype=np.float32)
        topk = np.empty(n, dtype=np.int32)
        seeds = np.empty(n, dtype=np.int64)
        rows = []  # (row, seq, allowed) for rows that need penalties or a token constraint
        known = None
        for i, s in enumerate(seqs):
            p = s.params
            temp[i] = p.temperature
            topp[i] = p.top_p
            topk[i] = p.top_k
            base = p.seed if p.seed is not None else (s.seq_id * 7919)
            seeds[i] = (base * 1000003 + len(s.output_ids)) & 0x7FFFFFFFFFFFFFFF
            allowed = None
            if p.allowed_tokens_fn is not None:
                # (a pending last token is speculated past by the constraint, ToolCallConstraint.__call__)
                allowed = p.allowed_tokens_fn(s.output_ids)
                f = spec_forced(allowed) if allowed is not None else None
                if f is not None:
                    known = known or {}
                    known[i] = f
            if allowed is not None or p.presence_penalty or p.frequency_penalty:
                rows.append((i, s, allowed))
        proc = upd = None
        if rows:
            proc, upd = self.lp.build(rows, n)
            upd = None if upd.empty else upd
        return SampleParams(temp, topp, topk, seeds, proc, not temp.any(), upd, known)

    def apply_proc_updates(self, sp: "SampleParams") -> None:
        """The step's logits-processor table writes, stream-ordered before its sampler (every TP rank)."""
        if sp.upd is not None:
            self.lp.apply(sp.upd, self._h2d)

    def proc_tables(self, sp: "SampleParams") -> dict:
        if sp.proc is None:
            return {}
        mask_tab, counts = self.lp.tables()
        return {"mask_tab": mask_tab, "counts": counts}

    def sample_device(self, logits: torch.Tensor, sp: "SampleParams") -> torch.Tensor:
        n = logits.shape[0]
        dev = logits.device
        pre, self._sp_dev = getattr(self, "_sp_dev", None), None
        if pre is not None and pre[0] is not sp:
            pre = None
        kw = self.proc_tables(sp)
        if sp.proc is not None:
            kw["proc"] = pre[4] if pre is not None and pre[4] is not None else self._h2d(sp.proc)
        if sp.greedy:
            return ops.sample(logits, torch.zeros(n, device=dev), **kw)
        if pre is not None and pre[2] is not None and pre[2].shape[0] == n:  # uploaded with the step's plan
            _, f32, tk, sd, _ = pre
            return ops.sample(logits, f32[:n], f32[n:], tk, sd, **kw)
        f32 = self._h2d(np.concatenate([sp.temp, sp.topp]))
        return ops.sample(logits, f32[:n], f32[n:], self._h2d(sp.topk), self._h2d(sp.seeds), **kw)

    # ------------------------------------------------------------------------------------------------------------
    @torch.inference_mode()
    def execute(self, batch: ScheduledBatch) -> tuple[list[Sequence], list[int]]:
        host, sample_seqs = self.build_host(batch)
        return sample_seqs, self.collect(self.launch(host, sample_seqs))

    @torch.inference_mode()
    def launch(self, host: HostStep, sample_seqs: list[Sequence], prev: Launched | None = None) -> Launched:
        """Enqueue one step on the GPU without waiting for it: (TP broadcast) -> H2D -> forward -> sample -> async
        D2H of the sampled ids into pinned memory. ``collect`` waits for them.

        Decode rows whose input token was PENDING at planning time are filled from the host if the token has landed
        since, else device-side from ``prev`` (the in-flight step that samples it): one gather + scatter on the
        stream, so the launch never waits for the previous step. Under TP the followers do the same from their own
        copy of the sampled ids (every rank samples the all-gathered logits with the same parameters)."""
        late_dst, late_src = [], []
        for row, s, pos in host.patch:
            t = s.token_at(pos)
            if t >= 0:
                host.i64[row] = t
            else:
                if prev is None or prev.rows is None or s.seq_id not in prev.rows:
                    raise RuntimeError(f"decode row {row}: token {pos} of seq {s.seq_id} is neither landed nor in "
                                       "the in-flight step")
                late_dst.append(row)
                late_src.append(prev.rows[s.seq_id])
        host.patch = []
        if late_dst:
            host.late_off, host.n_late = host.i64.size, len(late_dst)
            host.i64 = np.concatenate([host.i64, np.asarray(late_dst + late_src, dtype=np.int64)])
        self.last_stats = host.stats
        self.recent_stats.append(host.stats)
        self.rows_hist[bisect.bisect_left(ROWS_BUCKETS, host.T)] += 1
        sp = self.sample_params(sample_seqs)
        self.stager.begin()
        if self.broadcast is not None:  # TP leader: followers run the same step on their shards
            self.broadcast(host, sp)
        ev_s = None
        if self.step_events is not None and self.device.type == "cuda":
            ev_s = torch.cuda.Event(enable_timing=True)
            ev_s.record()
        toks = self._run(host, sp)
        rows = {s.seq_id: i for i, s in enumerate(sample_seqs)}
        if self.device.type != "cuda":
            return Launched(toks.clone(), None, toks, rows, known=sp.known)
        n = toks.shape[0]
        # a ring of pinned landing buffers: two steps can be in flight, each D2H needs its own
        ring = self._tok_host
        if ring is None or ring[0].shape[0] < n or ring[0].dtype != toks.dtype:
            ring = self._tok_host = [torch.empty(max(n, 256), dtype=toks.dtype, pin_memory=True) for _ in range(3)]
        self._tok_i = (getattr(self, "_tok_i", 0) + 1) % len(ring)
        out = ring[self._tok_i][:n]
        out.copy_(toks, non_blocking=True)
        err_idx = None
        car = self._custom_ar()
        if car is not None:  # the error word rides along with the sampled ids (4 bytes, same stream)
            if self._err_host is None:
                self._err_host = torch.zeros(len(ring), dtype=torch.int32, pin_memory=True)
            err_idx = self._tok_i
            car.error_async(self._err_host, err_idx)
        ev = torch.cuda.Event()
        ev.record()
        if ev_s is not None:  # GPU span of the step (plan upload -> token download), read back after the run
            ev_e = torch.cuda.Event(enable_timing=True)
            ev_e.record()
            self.step_events.append((ev_s, ev_e))
        return Launched(out, ev, toks, rows, err_idx, sp.known)

    def _custom_ar(self):
        """The IPC collective whose error word rides back with every step's ids: the TP group's custom all-reduce,
        or — data-parallel attention (tp = 1) — the EP group's IPC all-to-all (a peer that stops arriving makes its
        a2a waits time out; without this check the live ranks would stream tokens built from stale expert rows)."""
        if not hasattr(self, "_car"):
            from kafka_llm_service_amd.parallel import comm
            from kafka_llm_service_amd.parallel import state as pstate

            self._car = None
            if self.model.tp > 1:
                self._car = pstate.custom_ar()
            elif getattr(self.model, "dp_attention", False) and self.model.ep > 1 and self.device.type == "cuda":
                self._car = comm.get_custom(pstate.get().ep_group)
        return self._car

    @torch.inference_mode()
    def follower_launch(self, host: HostStep, sp: SampleParams) -> None:
        """A TP follower's copy of the leader's step (``tp_worker.follower_loop``): same forward on this rank's shard,
        same collectives, same sampler — nothing comes back to the host."""
        self.last_stats = host.stats
        self.stager.begin()
        self._run(host, sp)

    def _run(self, host: HostStep, sp: SampleParams) -> torch.Tensor:
        """Forward + sampling of one step (hipGraph replay for eligible decode steps): the sampled ids on the device,
        also left in ``tok_buf`` for the next step's late decode rows."""
        toks = None
        self.apply_proc_updates(sp)
        if self.graphs is not None and self.graphs.eligible(host, sp):
            toks = self.graphs.run(host, sp)
        if toks is None:
            inp = self.to_device(host, sp)
            logits = self.model.forward(inp, self.k_caches, self.v_caches)
            toks = self.sample_device(logits, sp)
            self.tok_buf[:toks.shape[0]].copy_(toks)
        return toks

    def collect(self, h: "Launched") -> list[int]:
        if h.event is not None:
            h.event.synchronize()
        if h.err_idx is not None and int(self._err_host[h.err_idx]) != 0:
            raise CollectiveError("custom all-reduce / all-to-all: a peer did not arrive within 2 s; failing the "
                                  "replica")
        return h.tokens.tolist()
