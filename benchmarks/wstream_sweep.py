#!/usr/bin/env python3
"""Configuration sweep of the weight-streaming decode GEMM (csrc/wstream_gemm.hip): for each Llama-3 projection
shape and decode batch M, time every (row tiles MT, K chunk KC, split count S) variant, with the cost of combining
the split-K slabs (``slab_reduce``) reported alongside. Used to pick the host plan (kafka_wstream_plan).
One JSON line per (shape, M, MT, KC, S)."""
from __future__ import annotations

import argparse
import json

import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import _ext

from wstream_bench import SHAPES, timeit  # noqa: E402

# (MT, KC, KW, PIN): PIN = weight prefetch pinned ahead of the MFMAs (wstream_gemm_kernel)
VARIANTS = [(mt, kc, kw, pin) for mt, kc, kw in ((1, 256, 1), (1, 256, 2), (2, 256, 1), (2, 256, 2), (3, 256, 1),
                                               (4, 128, 1), (4, 128, 2)) for pin in (0, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="16,64,128")
    ap.add_argument("--shapes", default="8b.qkv,8b.o,8b.gate_up,8b.down,8b.lm_head")
    ap.add_argument("--variants", default="", help="MT:KC:KW:PIN,... (default: all)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ext = _ext.load()
    for name in args.shapes.split(","):
        N, K = SHAPES[name]
        nbytes = N * K * 2
        copies = max(2, (600 << 20) // nbytes + 1)
        wts = [ops.tile_weight((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(copies)]
        for M in [int(m) for m in args.M.split(",")]:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            ref = x.float() @ ops.untile_weight(wts[0]).float().t()
            variants = ([tuple(int(v) for v in x.split(":")) for x in args.variants.split(",")] if args.variants
                        else VARIANTS)
            for mt, kc, kw, pin in variants:
                if M > 32 * mt:
                    continue
                for s in (1, 2, 4, 8):
                    if K % (kc * s):
                        continue
                    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                    p = torch.empty(s, M, N, device=dev) if s > 1 else None

                    def run(wt, y=y, p=p, mt=mt, kc=kc, s=s, kw=kw, pin=pin):
                        ext.wstream_gemm_cfg(x, wt, y if s == 1 else None, p, mt, kc, s, True, kw, pin)

                    t = timeit([lambda wt=wt: run(wt) for wt in wts])
                    t_red = timeit([lambda: ext.slab_reduce(p, y)]) if s > 1 else 0.0
                    run(wts[0])
                    if s > 1:
                        ext.slab_reduce(p, y)
                    err = (y.float() - ref).abs().max().item()
                    print(json.dumps({"shape": name, "M": M, "mt": mt, "kc": kc, "kw": kw, "pin": pin, "S": s,
                                      "us": round(t, 1),
                                      "TB/s": round(nbytes / t / 1e6, 2), "reduce_us": round(t_red, 1), "err": round(err, 4),
                                      "grid": ((N + 127) // 128) * s}), flush=True)
        del wts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
