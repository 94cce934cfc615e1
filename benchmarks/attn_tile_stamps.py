#!/usr/bin/env python3
"""Where a cascade tile-attention launch spends its time, per workgroup: the tile kernel's ABL = 8 diagnostic build
stamps the 100 MHz constant clock at entry, after the prologue (page ids staged, Q fragments loaded), when the first
64-key tile has landed, after the key loop and after the epilogue (csrc/attn_tile.hip). Same cascade shape as
benchmarks/attn_tile_anatomy.py (64 decode rows x Hq 32 / Hkv 8, D 128, an 18k-key prefix split into key chunks).
Prints one JSON line per chunk size: launch wall (events) and the phase medians / spreads in microseconds."""
from __future__ import annotations

import json
import os
import statistics

os.environ["KAFKA_TILE_ABL"] = "8"  # read once, at the first tile launch

import torch  # noqa: E402

from kafka_llm_service_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    Hq, Hkv, D, B = 32, 8, 128, 64
    G = Hq // Hkv
    torch.manual_seed(0)
    P = 18048
    n_pref = P // 16
    k = torch.randn(n_pref + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(n_pref + 8, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
    bt = torch.arange(n_pref + 4, dtype=torch.int32, device=dev).view(1, -1)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=dev)
    splits = 64
    part = torch.empty(B, Hq, splits, D, device=dev)
    lse = torch.zeros(B, Hq, splits, device=dev)
    tile = ops.tile_rows(3) // G
    for nk in (64, 192, 576, 1152, 2304):
        S = min(splits, P // nk, 32 if nk < 576 else splits)
        items = [(g0, min(tile, B - g0), 0, c * nk, (c + 1) * nk, c, 0, 0) for g0 in range(0, B, tile) for c in range(S)]
        it = torch.tensor(items, dtype=torch.int32, device=dev)
        nwg = len(items) * Hkv

        def fn():
            ops.attn_prefill(it, q, k, v, bt, q_limit, 0.088, out_part=part, lse_part=lse, variant=3)

        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        walls, ph = [], {"start_skew": [], "prologue": [], "first_tile": [], "loop": [], "epilogue": [],
                         "end_skew": [], "span": []}
        for _ in range(10):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            walls.append(s.elapsed_time(e) * 1e3)
            st = lse.view(-1).view(torch.int64)[:nwg * 8].view(nwg, 8)[:, :5].cpu().double() * 0.01  # us
            t0 = st[:, 0].min()
            ph["start_skew"].append(float((st[:, 0] - t0).max()))
            ph["prologue"].append(float((st[:, 1] - st[:, 0]).median()))
            ph["first_tile"].append(float((st[:, 2] - st[:, 1]).median()))
            ph["loop"].append(float((st[:, 3] - st[:, 2]).median()))
            ph["epilogue"].append(float((st[:, 4] - st[:, 3]).median()))
            ph["end_skew"].append(float(st[:, 4].max() - st[:, 4].min()))
            ph["span"].append(float(st[:, 4].max() - t0))
        rec = {"keys_per_wg": nk, "tiles_per_wg": nk // 64, "wgs": nwg, "wall_us": round(statistics.median(walls), 2)}
        rec.update({k2: round(statistics.median(v2), 2) for k2, v2 in ph.items()})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
