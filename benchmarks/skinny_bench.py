"""Skinny MFMA GEMM (csrc/skinny_gemm.hip) vs hipBLASLt (F.linear) on the Llama-3-8B projections at the row counts of
mixed decode + prefill steps (129..256), plus the streaming decode kernel at 128 rows for scale. One JSON line each."""
import json

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops


def timeit(fn, iters=30, rounds=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main():
    dev = "cuda"
    shapes = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
              ("down", 4096, 14336, False)]
    for name, N, K, glu in shapes:
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        wt = ops.tile_weight(w, glu=glu)
        for M in (130, 168, 200, 232, 256):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            t_blas = timeit(lambda: F.linear(x, w))
            t_sk = timeit(lambda: ops.linear_skinny(x, wt, glu=glu))
            S = ops.skinny_plan(M, N, K)
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "splits": S, "hipblaslt_us": round(t_blas, 1),
                              "skinny_us": round(t_sk, 1), "skinny_TB/s": round(N * K * 2 / t_sk / 1e6, 2),
                              "speedup": round(t_blas / t_sk, 2)}), flush=True)


if __name__ == "__main__":
    main()
