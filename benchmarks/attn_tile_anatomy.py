#!/usr/bin/env python3
"""Anatomy of the tile attention kernel on the cascade shape (64 decode rows x Hq 32 / Hkv 8, D 128): fixed
per-workgroup cost vs per-tile cost, and partial (fp32 O + lse) vs bf16 output epilogues. One process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24)."""
from __future__ import annotations

import argparse
import json
import os
import statistics

import torch

from kafka_llm_service_amd import ops


def timeit(fn, iters=20, rounds=5):
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,3")
    ap.add_argument("--keys", default="64,128,256,576,1152,2304")
    ap.add_argument("--splits", type=int, default=32)
    args = ap.parse_args()
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
    part = torch.empty(B, Hq, args.splits, D, device=dev)
    lse = torch.empty(B, Hq, args.splits, device=dev)
    out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
    for nk in [int(x) for x in args.keys.split(",")]:
        S = min(args.splits, P // nk)  # every item's key range inside the P staged prefix pages
        for var in [int(x) for x in args.variants.split(",")]:
            tile = ops.tile_rows(var) // G
            for mode in ("part", "bf16"):
                items = [(g0, min(tile, B - g0), 0, c * nk, (c + 1) * nk, c if mode == "part" else -1, 0, 0)
                         for g0 in range(0, B, tile) for c in range(S)]
                it = torch.tensor(items, dtype=torch.int32, device=dev)
                if mode == "part":
                    fn = lambda: ops.attn_prefill(it, q, k, v, bt, q_limit, 0.088, out_part=part,
                                                  lse_part=lse, variant=var)
                else:
                    fn = lambda: ops.attn_prefill(it, q, k, v, bt, q_limit, 0.088, out=out, variant=var)
                us = timeit(fn)
                flops = 4 * B * Hq * nk * S * D
                print(json.dumps({"keys_per_wg": nk, "slots": os.environ.get("KAFKA_TILE_SLOTS", "3"), "variant": var, "epilogue": mode, "wgs": len(items) * Hkv,
                                  "us": round(us, 2), "TF/s": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
