#!/usr/bin/env python3
"""Decode-shaped GEMMs of Llama-3-8B (y = x W^T, bf16): hipBLASLt vs rocBLAS vs bmm split-K vs the in-tree weight-streaming GEMM (csrc/wstream_gemm.hip).

Reports us/call and the weight-streaming bandwidth (weights are read once per call; x is tiny)."""
from __future__ import annotations

import json
import statistics
import sys

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=30, rounds=5):
    """fn(i) is called with the iteration index (used to rotate weight copies so every call streams from HBM)."""
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
    Ms = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,16,32,64,128").split(",")]
    libs_only = "--libs-only" in sys.argv  # TunableOp runs: plain F.linear only (strided bmm faults while tuning)
    dev = torch.device("cuda:0")
    have_custom = False
    try:
        from kafka_llm_service_amd import ops

        have_custom = hasattr(ops, "linear_stream")
    except Exception:
        pass
    for name, (N, K) in SHAPES.items():
        nrot = max(1, -(-640 * 2**20 // (N * K * 2)))  # > 256 MB Infinity Cache in total
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
        w = ws[0]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            row = {"gemm": name, "M": M, "N": N, "K": K}
            for lib in ("cublaslt", "cublas"):
                torch.backends.cuda.preferred_blas_library(lib)
                us = timeit(lambda i: F.linear(x, ws[i % nrot]))
                row[f"{'hipblaslt' if lib == 'cublaslt' else 'rocblas'}_us"] = round(us, 1)
            torch.backends.cuda.preferred_blas_library("cublaslt")
            for S in (() if libs_only else (2, 4, 8)):
                if K % S:
                    continue
                xs = x.view(M, S, K // S).transpose(0, 1)

                def f(i, S=S, xs=xs):
                    wv = ws[i % nrot].view(N, S, K // S).permute(1, 2, 0)  # [S, K/S, N]
                    return torch.bmm(xs, wv).sum(0)
                ref = F.linear(x, w).float()
                err = (f(0).float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                row[f"bmm_splitk{S}_us"] = round(timeit(f), 1)
                row[f"bmm_splitk{S}_err"] = round(err, 4)
            if have_custom and ops.stream_plan(M, N, K) is not None and not libs_only:
                ref = F.linear(x, w).float()
                wts = [ops.tile_weight(wi) for wi in ws]
                y = ops.slab_reduce(ops.linear_stream(x, wts[0]))
                err = (y.float() - ref).abs().max().item()
                row["wstream_us"] = round(timeit(lambda i: ops.linear_stream(x, wts[i % nrot])), 1)
                row["wstream_err"] = round(err / (ref.abs().max().item() + 1e-6), 4)
                del wts
            best = min(v for k, v in row.items() if k.endswith("_us"))
            row["best_TB/s"] = round(N * K * 2 / best / 1e6, 2)
            print(json.dumps(row), flush=True)
        del ws, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
