#!/usr/bin/env python3
"""Cascade prefix pass and suffix decode attention of one layer on the headline shape (64 rows, Llama-3-8B heads,
18k shared prefix, per-row suffixes of ~1.3k-4k keys), run three ways:

  seq       the engine's order today: prefix pass (bf16 partials) -> decode kernel (suffix + fused ticket merge)
  seq_fp32  as seq with fp32 prefix partials (the fused merge reads them as 16-B loads)
  seqsplit  prefix pass (fp32 partials) -> decode kernel (suffix partials only) -> attn_merge
  seqsplit_bf16  as seqsplit with the prefix partials in bf16 (attn_merge reads slots < npre from them)
  conc      prefix pass on a second stream CONCURRENT with the decode kernel (suffix partials), then attn_merge
  cascade / decode_fused / decode_part / merge   each launch of the above alone (inputs left by a previous run)

The prefix pass is a short-lived launch with fixed phases (prologue, first tile, epilogue) during which HBM idles;
the decode kernel is a long random-gather stream. Prints one JSON line per mode (us per layer) and the max abs
difference of each mode's output against ``seq``.
"""
from __future__ import annotations

import argparse
import json
import statistics

import numpy as np
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.model_runner import decode_items_fixed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--prefix", type=int, default=18000)
    ap.add_argument("--suffix-lo", type=int, default=1300)
    ap.add_argument("--suffix-hi", type=int, default=4000)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--chunks", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv, D, G = 32, 8, 128, 4
    B, P = args.B, args.prefix
    rng = np.random.default_rng(0)
    suffix = rng.integers(args.suffix_lo, args.suffix_hi + 1, B)
    lens = P + suffix
    n_pref = -(-P // 16)
    need = int(sum(-(-int(x) // 16) for x in suffix)) + n_pref + 8
    nb = need + 64
    maxb = int(lens.max()) // 16 + 2
    torch.manual_seed(0)
    caches = [(torch.randn(nb, Hkv, 16, D, device=dev, dtype=torch.bfloat16),
               torch.randn(nb, Hkv, D, 16, device=dev, dtype=torch.bfloat16)) for _ in range(args.layers)]
    bt = np.zeros((B, maxb), dtype=np.int32)
    free = rng.permutation(np.arange(n_pref, nb))
    c = 0
    for b in range(B):
        bt[b, :n_pref] = np.arange(n_pref)
        k = -(-int(suffix[b]) // 16)
        bt[b, n_pref:n_pref + k] = free[c:c + k]
        c += k
    btd = torch.from_numpy(bt).to(dev)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    scale = D ** -0.5
    npre = args.chunks
    ck = -(-P // (npre * 32)) * 32
    pit = [(0, B, 0, i * ck, min(P, (i + 1) * ck), i, 0, 0) for i in range(npre) if i * ck < P]
    npre = len(pit)
    pitd = torch.tensor(pit, dtype=torch.int32, device=dev)
    ditems = decode_items_fixed(lens.astype(np.int64), np.full(B, P, dtype=np.int64), np.full(B, npre), Hkv)
    real = ditems[:, 3] >= 0
    S = int((npre + ditems[real, 4]).max())
    dit = torch.from_numpy(ditems).to(dev)
    q_limit = torch.from_numpy(lens.astype(np.int32) - 1).to(dev)
    part = torch.empty(B, Hq, S, D, device=dev)
    lse = torch.full((B, Hq, S), float("-inf"), device=dev)
    pre = torch.empty(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
    outs = {m: torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16) for m in ("seq", "seq_fp32", "seqsplit", "seqsplit_bf16",
                                                                                   "conc")}
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def cascade(i, op, stream=None):
        kc, vc = caches[i % args.layers]
        ops.attn_prefill(pitd, q, kc, vc, btd, q_limit, scale, out_part=op, lse_part=lse, variant=3)

    def run(mode, i):
        kc, vc = caches[i % args.layers]
        if mode == "seq":
            cascade(i, pre)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale, out=outs[mode], pre_part=pre)
        elif mode == "seq_fp32":
            cascade(i, part)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale, out=outs[mode])
        elif mode == "seqsplit":
            cascade(i, part)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            ops.attn_merge(part, lse, outs[mode])
        elif mode == "seqsplit_bf16":
            cascade(i, pre)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            ops.attn_merge(part, lse, outs[mode], pre=pre, npre=npre)
        elif mode == "merge_bf16":
            ops.attn_merge(part, lse, outs["seqsplit_bf16"], pre=pre, npre=npre)
        elif mode == "cascade":
            cascade(i, pre)
        elif mode == "decode_fused":
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale, out=outs["seq"], pre_part=pre)
        elif mode == "decode_part":
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
        elif mode == "merge":
            ops.attn_merge(part, lse, outs["seqsplit"])
        else:
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                cascade(i, part)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            main_s.wait_stream(side)
            ops.attn_merge(part, lse, outs[mode])

    for mode in ("seq", "seq_fp32", "seqsplit", "seqsplit_bf16", "conc", "cascade", "decode_fused", "decode_part", "merge",
                 "merge_bf16"):
        res = []
        for _ in range(5):
            run(mode, 0)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(args.iters):
                run(mode, i)
            e.record()
            torch.cuda.synchronize()
            res.append(s.elapsed_time(e) * 1e3 / args.iters)
        run(mode, 0)
        torch.cuda.synchronize()
        err = (outs[mode].float() - outs["seq"].float()).abs().max().item() if mode in ("seq_fp32", "seqsplit", "seqsplit_bf16", "conc") \
            else 0.0
        print(json.dumps({"mode": mode, "us": round(statistics.median(res), 1), "S": S, "prefix_items": npre,
                          "decode_items": int(ditems.shape[0]), "err_vs_seq": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
