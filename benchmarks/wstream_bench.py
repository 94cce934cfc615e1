#!/usr/bin/env python3
"""Decode-GEMM microbenchmark: weight-streaming MFMA kernel on wave-tiled weights (csrc/wstream_gemm.hip) vs
hipBLASLt (torch F.linear) on the per-layer projection shapes of Llama-3-8B (TP=1) and Llama-3-70B (TP=8).

The streaming kernel's time includes what its consumer pays to combine split-K slabs only in the "+reduce" column
(the engine never runs that reduce: rope_kv / SwiGLU / add+RMSNorm sum the slabs while loading). Each case is a fresh
weight buffer larger than the Infinity Cache rotation (cold HBM reads, like one layer of a real step).
One JSON line per (shape, M)."""
from __future__ import annotations

import argparse
import json
import statistics

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops

SHAPES = {
    "8b.qkv": (6144, 4096), "8b.o": (4096, 4096), "8b.gate_up": (28672, 4096), "8b.down": (4096, 14336),
    "8b.lm_head": (128256, 4096),
    "70b-tp8.qkv": (1280, 8192), "70b-tp8.o": (8192, 1024), "70b-tp8.gate_up": (7168, 8192),
    "70b-tp8.down": (8192, 3584),
}


def timeit(fns, iters=20, rounds=5):
    """fns: list of callables, each touching its own weight copy (round-robin so every call reads cold-ish HBM)."""
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for f in fns:
            f()
        torch.cuda.synchronize()
        s.record()
        for i in range(iters):
            fns[i % len(fns)]()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="1,16,64,128")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, (600 << 20) // nbytes + 1)  # > 512 MB of weights in rotation: beyond the 256 MB MALL
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wts = [ops.tile_weight(w) for w in ws]
        for M in [int(m) for m in args.M.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            plan = ops.stream_plan(M, N, K)
            t_blas = timeit([lambda w=w: F.linear(x, w) for w in ws])
            row = {"shape": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_blas, 1),
                   "hipblaslt_TB/s": round(nbytes / t_blas / 1e6, 2)}
            if plan is not None:
                t_ws = timeit([lambda wt=wt: ops.linear_stream(x, wt) for wt in wts])
                t_ws1 = timeit([lambda wt=wt: ops.linear_stream(x, wt, max_splits=1) for wt in wts])
                t_red = timeit([lambda wt=wt: ops.slab_reduce(ops.linear_stream(x, wt)) for wt in wts])
                ref = x.float() @ ws[0].float().t()
                err = (ops.slab_reduce(ops.linear_stream(x, wts[0])).float() - ref).abs().max().item()
                row.update({"splits": plan[2], "wstream_us": round(t_ws, 1), "wstream_TB/s": round(nbytes / t_ws / 1e6, 2),
                            "wstream_s1_us": round(t_ws1, 1), "wstream+reduce_us": round(t_red, 1),
                            "speedup": round(t_blas / t_ws, 2), "max_err": round(err, 4)})
            print(json.dumps(row), flush=True)
        del ws, wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
