"""Skinny MFMA GEMM (csrc/skinny_gemm.hip) vs hipBLASLt (F.linear) vs the weight-streaming kernel as two 128-row
tiles (csrc/wstream_gemm.hip, pinned prefetch, best split) on the Llama-3-8B projections at the row counts of mixed
decode + prefill steps (129..256). Each timed call reads a different copy of the weight (>= 600 MB rotated, so the
MALL does not serve repeats). One JSON line each."""
import json

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops


def timeit(fn, iters=30, rounds=5):
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(iters):
            fn(i)
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / iters)
    return best


def main():
    dev = "cuda"
    shapes = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
              ("down", 4096, 14336, False)]
    ext = ops._ext.load()
    for name, N, K, glu in shapes:
        copies = max(2, (600 << 20) // (N * K * 2) + 1)
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        wts = [ops.tile_weight(w, glu=glu) for w in ws]
        for M in (130, 168, 200, 232, 256):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            t_blas = timeit(lambda i: F.linear(x, ws[i % copies]))
            t_sk = timeit(lambda i: ops.linear_skinny(x, wts[i % copies], glu=glu))
            S = ops.skinny_plan(M, N, K)
            best = None
            for s_ in (1, 2, 4, 8):
                if K % (128 * s_):
                    continue
                y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                p = torch.empty(s_, M, N, device=dev) if s_ > 1 else None
                for pin in (0, 1):
                    t = timeit(lambda i: ext.wstream_gemm_cfg(x, wts[i % copies], y if s_ == 1 else None, p, 4, 128,
                                                              s_, True, 1, pin))
                    t_red = timeit(lambda i: ext.slab_reduce(p, y)) if s_ > 1 else 0.0
                    if best is None or t + t_red < best[0]:
                        best = (t + t_red, s_, pin)
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "splits": S, "hipblaslt_us": round(t_blas, 1),
                              "skinny_us": round(t_sk, 1), "skinny_TB/s": round(N * K * 2 / t_sk / 1e6, 2),
                              "wstream_rt2_us": round(best[0], 1), "wstream_S": best[1], "wstream_pin": best[2],
                              "speedup": round(t_blas / t_sk, 2)}), flush=True)
        del ws, wts
        torch.cuda.empty_cache()

if __name__ == "__main__":
    main()
