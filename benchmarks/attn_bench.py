#!/usr/bin/env python3
"""Attention kernel microbenchmark on the bench.py shapes (Llama-3-8B heads: Hq 32, Hkv 8, D 128).

Cases (all in one process, interleaved rounds, median of N — cdna_hip_programming.md §5.4 rule 24):
  cascade   64 decode rows x 18,000-token shared prefix (prefix pass of cascade attention)
  decode    64 sequences x ~2,000-token private suffix (split-K decode)
  full      64 sequences x ~20,000 tokens without cascade (naive per-sequence decode)
  prefill   64-token new turn against a 20,000-token cached context (key-split tiles + merge)
  merge     [64, 32, S, 128] partial merge
Prints one JSON line per case with us/call and effective GB/s.
"""
from __future__ import annotations

import argparse
import json
import math
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
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--prefix", type=int, default=18000)
    ap.add_argument("--suffix", type=int, default=2000)
    ap.add_argument("--chunks", default="384,576,1024")
    ap.add_argument("--kv-dtype", default="bf16", choices=["bf16", "fp8"])
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv, D = 32, 8, 128
    G = Hq // Hkv
    tile = 128 // G
    B, P, Ls = args.B, args.prefix, args.suffix
    torch.manual_seed(0)
    n_pref = P // 16
    suf_pages = (Ls + 16) // 16 + 1
    nb = n_pref + B * suf_pages + 16
    if args.kv_dtype == "fp8":  # same random values, packed as e4m3 pages with per-token scales
        from kafka_llm_service_amd.ops import reference as ref

        k, v = ref.fp8_pack_pages(torch.randn(nb, Hkv, 16, D, device=dev), torch.randn(nb, Hkv, 16, D, device=dev))
    else:
        k = torch.randn(nb, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(nb, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
    maxb = n_pref + suf_pages + 2
    bt = torch.zeros(B + 1, maxb, dtype=torch.int32)
    c = n_pref
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        bt[b, n_pref:n_pref + suf_pages] = torch.arange(c, c + suf_pages)
        c += suf_pages
    bt = bt.to(dev)
    lens = torch.full((B,), P + Ls, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    q_limit = (lens - 1).to(torch.int32)
    scale = D ** -0.5
    out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
    kv_bytes_tok = Hkv * D * 2 * 2 if args.kv_dtype == "bf16" else Hkv * (2 * D + 2)

    # cascade prefix pass, several chunk sizes
    for chunk in [int(x) for x in args.chunks.split(",")]:
      nc = math.ceil(P / chunk)
      part = torch.empty(B, Hq, nc + 2, D, device=dev)
      lse = torch.empty(B, Hq, nc + 2, device=dev)
      for var in (0, 3):
        tile = ops.tile_rows(var) // G
        items = [(g0, min(tile, B - g0), 0, ci * chunk, min(P, (ci + 1) * chunk), ci, 0, 0)
                 for g0 in range(0, B, tile) for ci in range(nc)]
        it = torch.tensor(items, dtype=torch.int32, device=dev)
        if True:
            us = timeit(lambda: ops.attn_prefill(it, q, k, v, bt, q_limit, scale, out_part=part, lse_part=lse,
                                                 variant=var))
            flops = 4 * B * Hq * P * D
            print(json.dumps({"case": "cascade", "variant": var, "chunk": chunk, "splits": nc,
                              "wgs": len(items) * Hkv, "us": round(us, 1), "TF/s": round(flops / us / 1e6, 1),
                              "GB/s_hbm": round(P * kv_bytes_tok / us / 1e3, 1)}))
      mus = timeit(lambda: ops.attn_merge(part, lse, out))
      print(json.dumps({"case": "merge", "S": nc + 2, "us": round(mus, 1),
                        "GB/s": round(part.numel() * 4 / mus / 1e3, 1)}))

    # decode over the suffix only (cascade second pass) and over the full context (no cascade)
    ks = torch.full((B,), P, dtype=torch.int32, device=dev)
    for S in (1, 2, 4):
        part = torch.empty(B, Hq, S, D, device=dev)
        lse = torch.empty(B, Hq, S, device=dev)
        it = ops.uniform_decode_items(lens, ks, S, 0)  # built once: the engine plans items on the host
        us = timeit(lambda: ops.attn_decode_items(q, k, v, bt, it, part, lse, scale))
        print(json.dumps({"case": "decode_suffix", "S": S, "us": round(us, 1),
                          "GB/s": round(B * Ls * kv_bytes_tok / us / 1e3, 1)}))
    for S in (4, 8, 16):
        part = torch.empty(B, Hq, S, D, device=dev)
        lse = torch.empty(B, Hq, S, device=dev)
        it = ops.uniform_decode_items(lens, None, S, 0)
        us = timeit(lambda: ops.attn_decode_items(q, k, v, bt, it, part, lse, scale), iters=5)
        print(json.dumps({"case": "decode_full", "S": S, "us": round(us, 1),
                          "GB/s_logical": round(B * (P + Ls) * kv_bytes_tok / us / 1e3, 1)}))

    # new-turn prefill: 64 tokens against the full context of sequence 0
    T = 64
    qp = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
    ctx = P + Ls - T
    ql = torch.arange(ctx, ctx + T, dtype=torch.int32, device=dev)
    for var in (0, 3):
        tile = ops.tile_rows(var) // G
        for ck in (1024, 2048, 4096, 0):
            if ck == 0:
                items = [(t0, min(tile, T - t0), 0, 0, ctx + T, -1, 0, 0) for t0 in range(0, T, tile)]
                it = torch.tensor(items, dtype=torch.int32, device=dev)
                o = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
                us = timeit(lambda: ops.attn_prefill(it, qp, k, v, bt, ql, scale, out=o, variant=var), iters=5)
            else:
                ns = math.ceil((ctx + T) / ck)
                items = [(t0, min(tile, T - t0), 0, c0 * ck, min(ctx + T, (c0 + 1) * ck), c0, 0, 0)
                         for t0 in range(0, T, tile) for c0 in range(ns)]
                it = torch.tensor(items, dtype=torch.int32, device=dev)
                part = torch.empty(T, Hq, ns, D, device=dev)
                lse = torch.full((T, Hq, ns), float("-inf"), device=dev)
                o = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)

                def f():
                    ops.attn_prefill(it, qp, k, v, bt, ql, scale, out_part=part, lse_part=lse, variant=var)
                    ops.attn_merge(part, lse, o)
                us = timeit(f, iters=5)
            print(json.dumps({"case": "prefill_newturn", "variant": var, "kv_chunk": ck, "us": round(us, 1)}))

    # cold prefill throughput: 2048-token chunk at the start of a sequence (causal)
    T = 2048
    qp = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
    ql = torch.arange(0, T, dtype=torch.int32, device=dev)
    o = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
    for var in (0, 3):
        tile = ops.tile_rows(var) // G
        items = [(t0, min(tile, T - t0), 0, 0, t0 + tile, -1, 0, 0) for t0 in range(0, T, tile)]
        it = torch.tensor(items, dtype=torch.int32, device=dev)
        us = timeit(lambda: ops.attn_prefill(it, qp, k, v, bt, ql, scale, out=o, variant=var), iters=5)
        flops = 2 * T * T * Hq * D  # causal: half of 4*T*T*Hq*D
        print(json.dumps({"case": "prefill_causal_2k", "variant": var, "us": round(us, 1),
                          "TF/s": round(flops / us / 1e6, 1)}))
    # the engine's plan (model_runner.plan_prefill_items): long tiles split into key pieces + per-range merges
    from kafka_llm_service_amd.engine.model_runner import plan_prefill_items

    for var, T in [(v_, t_) for v_ in (0, 3) for t_ in (2048, 4096, 8192)]:
        qp = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
        ql = torch.arange(0, T, dtype=torch.int32, device=dev)
        o = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
        tile = ops.tile_rows(var) // G
        tiles = [(t0, min(tile, T - t0), 0, t0 + min(tile, T - t0), T) for t0 in range(0, T, tile)]
        items, splits, ranges = plan_prefill_items(tiles, Hkv, 256, 256)
        it = torch.tensor(items, dtype=torch.int32, device=dev)
        part = torch.empty(T, Hq, max(splits, 1), D, device=dev)
        lse = torch.full((T, Hq, max(splits, 1)), float("-inf"), device=dev)

        def fp():
            ops.attn_prefill(it, qp, k, v, bt, ql, scale, out=o, out_part=part, lse_part=lse, variant=var)
            for lo, hi in ranges:
                ops.attn_merge(part[lo:hi], lse[lo:hi], o[lo:hi])
        us = timeit(fp, iters=5)
        flops = 2 * T * T * Hq * D
        print(json.dumps({"case": "prefill_causal_planned", "variant": var, "T": T, "splits": splits, "items": len(items),
                          "us": round(us, 1), "TF/s": round(flops / us / 1e6, 1)}))


if __name__ == "__main__":
    main()
