"""hipBLASLt default heuristic vs PyTorch TunableOp's tuned pick for the mixed-step gate_up (M = 129..256 rows,
N = 28672, K = 4096) and a few prefill shapes: us per call, weights rotated over >= 600 MB (cold in the MALL).
Run twice: once plain, once with PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 (it tunes each new shape
on its first call, then uses the pick). One JSON line per shape."""
import json
import os
import time

import torch
import torch.nn.functional as F


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
    tuned = os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1"
    for N, K, Ms in ((28672, 4096, (136, 168, 200, 232, 256)), (6144, 4096, (512, 1024)), (4096, 14336, (512, 1024))):
        copies = max(2, (600 << 20) // (N * K * 2) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for M in Ms:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            t0 = time.perf_counter()
            F.linear(x, ws[0])  # (tunes here when tuning is on)
            torch.cuda.synchronize()
            first = time.perf_counter() - t0
            us = timeit(lambda i: F.linear(x, ws[i % copies]))
            print(json.dumps({"tunableop": tuned, "M": M, "N": N, "K": K, "us": round(us, 1),
                              "TB/s": round(N * K * 2 / us / 1e6, 2), "first_call_s": round(first, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
