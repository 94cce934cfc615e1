#!/usr/bin/env python3
"""Offline PyTorch TunableOp pass over the hipBLASLt GEMM shapes of mixed decode+prefill steps (Llama-3-8B, bf16,
y = x W^T via F.linear). Result (profiles/r02/tunableop_mixed_step_gemms_rejected.log): across all hipBLASLt +
rocBLAS solutions nothing beats the library's default pick at these shapes (tuned = default within noise, several
worse), so the engine does not load a tuning file.

Mixed steps (64 decode rows + a new turn's prompt tokens, 129..256 rows padded to 16 k + 8 by
``model_runner.pad_step_rows``) are ~20 % of the headline bench's steps and their four projections on hipBLASLt's
default picks take ~167 us per layer (profiles/r02/kernel breakdown). For each shape this prints the default time,
tunes (all hipBLASLt + rocBLAS solutions, cold weights: copies rotated past the 256 MB MALL), and prints the tuned
time. Usage: python scripts/tune_gemm.py --ms 168,184,200,216,232,248 --out <csv>
"""
from __future__ import annotations

import argparse
import json
import os
import statistics

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="168,184,200,216,232,248")
    ap.add_argument("--out", required=True)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "40")
    import torch
    import torch.nn.functional as F

    tun = torch.cuda.tunable
    dev = torch.device("cuda:0")
    tun.set_filename(args.out, insert_device_ordinal=False)
    if os.path.exists(args.out):
        tun.read_file(args.out)

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

    Ms = [int(m) for m in args.ms.split(",")]
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        nrot = max(1, -(-640 * 2**20 // (N * K * 2)))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) for _ in range(nrot)]
        for M in Ms:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            tun.enable(False)
            base = timeit(lambda i: F.linear(x, ws[i % nrot]))
            ref = F.linear(x, ws[0]).float()
            tun.enable(True)
            tun.tuning_enable(True)
            F.linear(x, ws[0])  # tunes this shape (once)
            torch.cuda.synchronize()
            tun.tuning_enable(False)
            tuned = timeit(lambda i: F.linear(x, ws[i % nrot]))
            err = (F.linear(x, ws[0]).float() - ref).abs().max().item()
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "default_us": round(base, 1),
                              "tuned_us": round(tuned, 1), "max_abs_diff": err}), flush=True)
        del ws
        torch.cuda.empty_cache()
    # (TunableOp writes the results file itself at process exit while tuning is on)


if __name__ == "__main__":
    main()
