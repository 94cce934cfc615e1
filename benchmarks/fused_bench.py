#!/usr/bin/env python3
"""Fused decode-layer GEMM epilogues (csrc/wstream_gemm.hip FIN_*) vs the unfused kernel pairs they replace, on the
Llama-3-8B decode shapes, plus a per-workgroup phase anatomy of each fused launch from its 100 MHz stamps.

  o / down  : FIN_RES  vs  linear_stream (slabs) + fused_add_rmsnorm
  qkv       : FIN_ROPE vs  linear_stream (slabs) + rope_kv_write
  gate_up   : FIN_GLU  vs  linear_glu (fused SwiGLU, no row scale)
Weights rotate through > 512 MB of copies (cold HBM, like one layer of a real step). One JSON line per case; the
anatomy line gives medians over workgroups (us): loop = stream + MFMAs, drain = slab stores reaching the coherent
level, tail = from the last workgroup's main-loop end to the last finisher's end (what the fused epilogue adds to
the launch), fin = a finisher's body."""
from __future__ import annotations

import argparse
import json
import statistics

import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import reference as ref

SHAPES = {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096), "gate_up": (28672, 4096)}


def timeit(fns, iters=60, rounds=5):
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for f in fns[:2]:
            f()
        torch.cuda.synchronize()
        s.record()
        for i in range(iters):
            fns[i % len(fns)]()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def anatomy(st: torch.Tensor, grid: int) -> dict:
    t = st[:grid].cpu().double() / 100.0  # us
    t0 = t[:, 0].min()
    t = t - t0
    loop = (t[:, 1] - t[:, 0])
    done1 = t[:, 1]
    drain = (t[:, 2] - t[:, 1])[t[:, 2] > 0]
    fin = t[:, 4] > 0
    out = {"loop_med": float(loop.median()), "loop_max": float(loop.max()), "last_loop_end": float(done1.max()),
           "first_loop_end": float(done1.min())}
    if drain.numel():
        out["drain_med"] = float(drain.median())
    if fin.any():
        out["ticket_med"] = float((t[fin, 3] - t[fin, 2]).median())
        out["fin_med"] = float((t[fin, 4] - t[fin, 3]).median())
        out["end"] = float(t[fin, 4].max())
        out["tail"] = float(t[fin, 4].max() - done1.max())
    return {k: round(v, 2) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=64)
    ap.add_argument("--shapes", default="o,down,qkv,gate_up")
    ap.add_argument("--max-splits", default="8", help="comma list: split caps of the fused o / down / qkv launches")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    ext = ops._ext.load()
    M, eps, Hq, Hkv = args.M, 1e-5, 32, 8
    d = 4096
    resid = torch.randn(M, d, device=dev, dtype=torch.bfloat16)
    nw = torch.ones(d, device=dev, dtype=torch.bfloat16)
    xn = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    ss = torch.rand(d // 128, M, device=dev) * 100
    cs = ref.rope_cos_sin(32768, 128, 500000.0).to(dev)
    pos = torch.randint(0, 20000, (M,), device=dev)
    kc = torch.zeros(4096, Hkv, 16, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(4096, Hkv, 128, 16, device=dev, dtype=torch.bfloat16)
    slots = torch.randperm(4096 * 16, device=dev)[:M]
    q = torch.empty(M, Hq, 128, device=dev, dtype=torch.bfloat16)
    for name, ms in [(n, int(m)) for n in args.shapes.split(",") for m in args.max_splits.split(",")]:
        N, K = SHAPES[name]
        if name == "gate_up" and ms != 8:
            continue
        copies = max(2, (600 << 20) // (N * K * 2) + 1)
        glu = name == "gate_up"
        wts = [ops.tile_weight((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16), glu=glu)
               for _ in range(copies)]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        mt, kc_, S = ops.stream_plan(M, N, K, 1 if glu else ms)
        if name in ("o", "down"):
            def plain(wt):
                ops.fused_add_rmsnorm(ops.linear_stream(x, wt), resid, nw, eps, out=xn)

            def fused(wt, st=None):
                p = torch.empty(S, M, N, device=dev) if S > 1 else None
                ext.wstream_fin(1, x, wt, None, p, ops._tickets(dev, 64, "bench"), None, eps, resid, nw, xn, ss,
                                None, None, None, None, None, None, 0, 0, ms, st)
        elif name == "qkv":
            def plain(wt):
                ops.rope_kv_write(ops.linear_stream(x, wt), pos, cs, q, kc, vc, slots, Hq, Hkv)

            def fused(wt, st=None):
                p = torch.empty(S, M, N, device=dev) if S > 1 else None
                ext.wstream_fin(2, x, wt, None, p, ops._tickets(dev, 64, "bench"), ss, eps, None, None, None, None,
                                pos, cs, q, kc, vc, slots, Hq, Hkv, ms, st)
        else:
            def plain(wt):
                ops.linear_glu(x, wt)

            def fused(wt, st=None):
                y = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                ext.wstream_fin(3, x, wt, y, None, ops._tickets(dev, 64, "bench"), ss, eps, None, None, None, None,
                                None, None, None, None, None, None, 0, 0, 1, st)
        t_plain = timeit([lambda w=w: plain(w) for w in wts])
        t_gemm = timeit([lambda w=w: ops.linear_stream(x, w, 1 if glu else ms, glu=glu) for w in wts])
        t_fused = timeit([lambda w=w: fused(w) for w in wts])
        grid = (N // 128) * S
        st = torch.zeros(grid * 8 + 8, dtype=torch.long, device=dev)
        an = []
        for i in range(5):
            st.zero_()
            fused(wts[i % len(wts)], st)
            torch.cuda.synchronize()
            an.append(anatomy(st.view(-1, 8), grid))
        med = {k: round(statistics.median(a[k] for a in an if k in a), 2) for k in an[-1]}
        if glu:
            med = {}
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "splits": S, "plain_us": round(t_plain, 2),
                          "gemm_only_us": round(t_gemm, 2), "fused_us": round(t_fused, 2), "anatomy": med}),
              flush=True)


if __name__ == "__main__":
    main()
