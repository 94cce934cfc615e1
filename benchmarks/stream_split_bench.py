#!/usr/bin/env python3
"""Mixed-step GEMMs (129..256 rows, Llama-3-8B shapes): hipBLASLt on all rows vs the weight-streaming kernel run on
two row halves back to back (the second half's weight stream can hit the 256 MB MALL). Weights rotated over copies
so each measured call starts cold."""
import json
import statistics

import torch
import torch.nn.functional as F

from kafka_llm_service_amd import ops

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


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
    dev = torch.device("cuda:0")
    for name, (N, K) in SHAPES.items():
        nrot = max(2, -(-640 * 2**20 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(nrot)]
        wts = [ops.tile_weight(w) for w in ws]
        for M in (168, 200, 248):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            h = M // 2
            blas = timeit(lambda i: F.linear(x, ws[i % nrot]))
            two = timeit(lambda i: (ops.linear_stream(x[:h], wts[i % nrot]), ops.linear_stream(x[h:], wts[i % nrot])))
            one128 = timeit(lambda i: ops.linear_stream(x[:128], wts[i % nrot]))
            tiled = timeit(lambda i: ops.linear_stream(x, wts[i % nrot]))  # one launch, 2 row tiles per slice
            print(json.dumps({"gemm": name, "M": M, "hipblaslt_us": round(blas, 1), "stream_two_halves_us": round(two, 1),
                              "stream_128_rows_us": round(one128, 1), "stream_row_tiles_us": round(tiled, 1)}),
                  flush=True)
        del ws, wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
