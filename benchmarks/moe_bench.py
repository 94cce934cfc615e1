#!/usr/bin/env python3
"""Mixtral-8x7B MoE layer microbenchmark on one MI355X: router (HIP) + grouped gate_up GEMM + SiLU*mul + grouped
down GEMM with the fused weighted combine, at decode-like token counts (BASELINE config 5: 128 threads) and a
prefill chunk. Reports us/layer and the expert-weight streaming rate (every expert with >= 1 token is read once) for
the LDS-tiled grouped GEMM and, at decode sizes (T <= 128), for the grouped weight-streaming kernel.

  python benchmarks/moe_bench.py            # T = 1, 16, 64, 128, 512, 2048
"""
from __future__ import annotations

import json
import statistics
import sys

import torch

from kafka_llm_service_amd import ops


def timeit(fn, iters=20, rounds=5):
    res = []
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def main():
    Ts = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,16,64,128,512,2048").split(",")]
    dev = torch.device("cuda:0")
    E, K, d, F = 8, 2, 4096, 14336
    torch.manual_seed(0)
    router = (torch.randn(E, d, device=dev) * d ** -0.5).to(torch.bfloat16)
    w13 = (torch.randn(E, 2 * F, d, device=dev) * d ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, device=dev) * F ** -0.5).to(torch.bfloat16)
    w13t, w2t = ops.tile_experts(w13, glu=True), ops.tile_experts(w2)  # grouped weight-streaming layout
    for T in Ts:
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)

        def layer():
            r = ops.moe_route(torch.nn.functional.linear(x, router), K)
            h = ops.grouped_gemm(x, w13, r, gather=True)
            a = ops.silu_mul(h)
            out = torch.zeros(T, d, dtype=torch.float32, device=dev)
            ops.grouped_gemm(a, w2, r, gather=False, combine_out=out)
            return out

        def layer_stream():
            r = ops.moe_route(torch.nn.functional.linear(x, router), K)
            a = ops.grouped_stream_glu(x, w13t, r)
            out = torch.zeros(T, d, dtype=torch.float32, device=dev)
            ops.grouped_stream_combine(a, w2t, r, T, out)
            return out

        us = timeit(layer)
        us_s = timeit(layer_stream) if T <= 512 else None
        us_u = None
        if us_s:  # the grouped streaming kernel without the pinned prefetch (A/B of ops.GROUPED_PIN)
            ops.GROUPED_PIN = False
            us_u = timeit(layer_stream)
            ops.GROUPED_PIN = True
        r = ops.moe_route(torch.nn.functional.linear(x, router), K)
        used = int((r.expert_off[1:] - r.expert_off[:-1] > 0).sum().item())
        bytes_w = used * (2 * F * d + d * F) * 2
        print(json.dumps({"T": T, "experts_used": used, "us_per_layer": round(us, 1),
                          "weight_TB/s": round(bytes_w / us / 1e6, 2),
                          "TFLOP/s": round(2 * T * K * 3 * F * d / us / 1e6, 1),
                          "stream_us_per_layer": round(us_s, 1) if us_s else None,
                          "stream_weight_TB/s": round(bytes_w / us_s / 1e6, 2) if us_s else None,
                          "stream_unpinned_us_per_layer": round(us_u, 1) if us_u else None}), flush=True)


if __name__ == "__main__":
    main()
