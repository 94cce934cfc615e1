#!/usr/bin/env python3
"""Does the Infinity Cache (MALL, 256 MB) serve a decode GEMM's weights when they were read shortly before?

For the Llama-3-8B gate_up (28672 x 4096, fused SwiGLU) and o (4096 x 4096) projections at 64 rows, times the
weight-streaming GEMM (GEMM alone, events around it) when its weight copy is:
  cold      one of >= 4 rotated copies (> 900 MB between two reads of a copy)
  hot       the same copy as the previous call
  pref      read in full (a reduction over it) right before the GEMM
  pref_ev   read in full, then `--evict-mb` of other data streamed, then the GEMM (the suffix decode's KV stream
            sits between the cascade and the MLP in a decode layer)
  pref_part the first `--part` fraction of the copy read right before the GEMM
One JSON line per (projection, mode)."""
from __future__ import annotations

import argparse
import json
import statistics

import torch

from kafka_llm_service_amd import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--evict-mb", type=int, default=350)
    ap.add_argument("--part", type=float, default=0.5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = (torch.randn(args.M, 4096, device=dev) * 0.5).to(torch.bfloat16)
    ev_buf = torch.empty(args.evict_mb << 18, device=dev, dtype=torch.float32).normal_()
    sink = torch.empty(1, device=dev, dtype=torch.float32)

    def read_all(t: torch.Tensor, frac: float = 1.0):
        flat = t.view(-1).view(torch.float32)  # (bit patterns summed: only the read matters)
        sink.add_(flat[:int(flat.numel() * frac)].sum())

    for name, N, glu in (("gate_up", 28672, True), ("o", 4096, False)):
        copies = max(4, (1000 << 20) // (N * 4096 * 2) + 1)
        wts = [ops.tile_weight((torch.randn(N, 4096, device=dev) * 0.02).to(torch.bfloat16), glu=glu)
               for _ in range(copies)]
        gemm = (lambda w: ops.linear_glu(x, w)) if glu else (lambda w: ops.linear_stream(x, w))
        for _ in range(3):
            gemm(wts[0])
        torch.cuda.synchronize()
        for mode in ("cold", "hot", "pref", "pref_ev", "pref_part"):
            ts = []
            for i in range(args.iters):
                w = wts[0] if mode == "hot" else wts[i % copies]
                if mode in ("pref", "pref_ev"):
                    read_all(w)
                if mode == "pref_part":
                    read_all(w, args.part)
                if mode == "pref_ev":
                    read_all(ev_buf)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                gemm(w)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            print(json.dumps({"gemm": name, "M": args.M, "mode": mode, "us_median": round(statistics.median(ts), 1),
                              "us_min": round(min(ts), 1), "MB": round(N * 4096 * 2 / 2**20, 1),
                              "evict_mb": args.evict_mb if mode == "pref_ev" else 0,
                              "part": args.part if mode == "pref_part" else 1.0}), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
