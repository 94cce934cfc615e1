#!/usr/bin/env python3
"""Suffix decode attention on the headline shape (bench.py: Llama-3-8B heads Hq 32 / Hkv 8 / D 128, 64 rows, per-row
suffixes of ~1.3k-4k keys behind an 18k cascade prefix whose 32 bf16 partials per row are merged in the epilogue).

The work items are the engine's own (model_runner.decode_items at its 1344-workgroup target). Each layer has its own
K/V pool of ``--pool-blocks`` pages so consecutive calls do not re-read the Infinity Cache, and the suffix pages are
laid out either contiguous per row or scattered over the pool (what a long-running engine's free list hands out).
Prints one JSON line per (kernel, layout): us per call and the effective HBM rate of the suffix K/V bytes.
"""
from __future__ import annotations

import argparse
import json
import statistics

import numpy as np
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.model_runner import decode_items, decode_items_fixed


def timeit(fn, iters=20, rounds=5):
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn(0)
        torch.cuda.synchronize()
        s.record()
        for i in range(iters):
            fn(i)
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--prefix", type=int, default=18000)
    ap.add_argument("--suffix-lo", type=int, default=1300)
    ap.add_argument("--suffix-hi", type=int, default=4000)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--pool-blocks", type=int, default=40000)
    ap.add_argument("--npre", type=int, default=32)
    ap.add_argument("--targets", default="1344", help="decode workgroup targets to sweep (items x Hkv)")
    ap.add_argument("--layouts", default="contiguous,scattered")
    ap.add_argument("--plans", default="adaptive,fixed")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv, D = 32, 8, 128
    B, P = args.B, args.prefix
    rng = np.random.default_rng(0)
    suffix = rng.integers(args.suffix_lo, args.suffix_hi + 1, B)
    lens = P + suffix
    n_pref = P // 16
    maxb = int(lens.max()) // 16 + 2
    nb = args.pool_blocks
    torch.manual_seed(0)
    caches = [(torch.randn(nb, Hkv, 16, D, device=dev, dtype=torch.bfloat16),
               torch.randn(nb, Hkv, D, 16, device=dev, dtype=torch.bfloat16)) for _ in range(args.layers)]
    need = int(sum(-(-int(x) // 16) for x in suffix)) + n_pref + 8
    assert need <= nb, (need, nb)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    npre = np.full(B, args.npre)
    kv_start = np.full(B, P)
    plans = {}
    for t in (int(x) for x in args.targets.split(",")):
        if "adaptive" in args.plans:
            plans[f"adaptive{t}"] = decode_items(lens.astype(np.int64), kv_start.astype(np.int64), npre, Hkv,
                                                 target=t)
        if "fixed" in args.plans:
            plans[f"fixed{t}"] = decode_items_fixed(lens.astype(np.int64), kv_start.astype(np.int64), npre, Hkv,
                                                    target=t)
    S = 64
    part = torch.empty(B, Hq, S, D, device=dev)
    lse = torch.randn(B, Hq, S, device=dev) - 40.0  # prefix partials count, suffix dominates
    pre = torch.randn(B, Hq, S, D, device=dev).to(torch.bfloat16)
    out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
    suffix_bytes = int(suffix.sum()) * Hkv * D * 2 * 2
    for layout in args.layouts.split(","):
        bt = np.zeros((B, maxb), dtype=np.int32)
        free = np.arange(n_pref, nb)
        if layout == "scattered":
            free = rng.permutation(free)
        c = 0
        for b in range(B):
            bt[b, :n_pref] = np.arange(n_pref)
            k = -(-int(suffix[b]) // 16)
            bt[b, n_pref:n_pref + k] = free[c:c + k]
            c += k
        btd = torch.from_numpy(bt).to(dev)
        for pname, plan in plans.items():
            items = torch.from_numpy(plan).to(dev)
            fn = lambda i, items=items: ops.attn_decode_items(q, *caches[i % args.layers], btd, items, part, lse,  # noqa: E731
                                                                scale, out=out, pre_part=pre)
            us = timeit(fn)
            print(json.dumps({"kernel": "decode", "plan": pname, "layout": layout, "items": int(items.shape[0]),
                              "us": round(us, 1), "TB/s": round(suffix_bytes / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
