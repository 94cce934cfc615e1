#!/usr/bin/env python3
"""Cascade prefix pass and suffix decode attention of one layer on the headline shape (64 rows, Llama-3-8B heads,
18k shared prefix, per-row suffixes of ~1.3k-4k keys), run three ways:

  seq       the engine's order today: prefix pass (bf16 partials) -> decode kernel (suffix + fused ticket merge)
  seq_fp32  as seq with fp32 prefix partials (the fused merge reads them as 16-B loads)
  seqsplit  prefix pass (fp32 partials) -> decode kernel (suffix partials only) -> attn_merge
  seqsplit_bf16  as seqsplit with the prefix partials in bf16 (attn_merge reads slots < npre from them)
  conc      prefix pass on a second stream CONCURRENT with the decode kernel (suffix partials), then attn_merge
  cumask    as conc, but on two CU-MASKED streams (hipExtStreamCreateWithCUMask): the prefix pass on --cascade-cus
            CUs, the decode kernel on the other ones (no co-residency: each kernel keeps its own CUs), then attn_merge
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
    ap.add_argument("--cascade-cus", type=str, default="96,112,128",
                    help="cumask modes: CUs (of 256) given to the prefix pass")
    ap.add_argument("--mask-order", choices=("stripe", "block"), default="stripe",
                    help="stripe: CU-mask bits taken round-robin (bit i, i + 8, ...); block: the lowest bits")
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
    masked = {}  # C -> (cascade stream, decode stream)

    def cu_streams(C):
        if C not in masked:
            import ctypes
            # the HIP runtime torch already loaded (a second copy would not know torch's device context)
            libs = [ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64.so" in ln]
            hip = ctypes.CDLL(libs[0] if libs else "libamdhip64.so")
            ncu = torch.cuda.get_device_properties(dev).multi_processor_count
            if args.mask_order == "stripe":
                # bit i = (a, b, c) = (i // 32, i // 8 % 4, i % 8): whether a bit's XCD is i % 8 or i // 32, taking
                # (a + c) % 8 < k plus b < j where it equals k gives every XCD C / 8 CUs (C = 32 k + 8 j)
                k, j = C // 32, (C % 32) // 8
                sel = set(i for i in range(ncu) if ((i // 32 + i % 8) % 8 < k) or
                          ((i // 32 + i % 8) % 8 == k and (i // 8) % 4 < j))
            else:
                sel = set(range(C))
            words = []
            for which in (sel, set(range(ncu)) - sel):
                m = [0] * ((ncu + 31) // 32)
                for i in which:
                    m[i // 32] |= 1 << (i % 32)
                words.append(m)
            out = []
            for m in words:
                st = ctypes.c_void_p()
                arr = (ctypes.c_uint32 * len(m))(*m)
                rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), len(m), arr)
                assert rc == 0, f"hipExtStreamCreateWithCUMask: {rc}"
                out.append(torch.cuda.ExternalStream(st.value, device=dev))
            masked[C] = tuple(out)
        return masked[C]

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
        elif mode.startswith("cumask"):
            C = int(mode[6:])
            sa, sb = cu_streams(C)
            sa.wait_stream(main_s)
            sb.wait_stream(main_s)
            with torch.cuda.stream(sa):
                cascade(i, pre)
            with torch.cuda.stream(sb):
                ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            main_s.wait_stream(sa)
            main_s.wait_stream(sb)
            ops.attn_merge(part, lse, outs["conc"], pre=pre, npre=npre)
        elif mode.startswith("cascade_cu"):  # the prefix pass alone on its masked stream
            sa, _ = cu_streams(int(mode[10:]))
            sa.wait_stream(main_s)
            with torch.cuda.stream(sa):
                cascade(i, pre)
            main_s.wait_stream(sa)
        elif mode.startswith("decode_cu"):  # the decode kernel alone on the complement
            _, sb = cu_streams(int(mode[9:]))
            sb.wait_stream(main_s)
            with torch.cuda.stream(sb):
                ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            main_s.wait_stream(sb)
        else:
            side.wait_stream(main_s)
            with torch.cuda.stream(side):
                cascade(i, part)
            ops.attn_decode_items(q, kc, vc, btd, dit, part, lse, scale)
            main_s.wait_stream(side)
            ops.attn_merge(part, lse, outs[mode])

    cus = [int(x) for x in args.cascade_cus.split(",") if x]
    modes = ["seq", "seq_fp32", "seqsplit", "seqsplit_bf16", "conc", "cascade", "decode_fused", "decode_part", "merge",
             "merge_bf16"]
    for C in cus:
        modes += [f"cascade_cu{C}", f"decode_cu{C}", f"cumask{C}"]
    for mode in modes:
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
        om = "conc" if mode.startswith("cumask") else mode
        err = (outs[om].float() - outs["seq"].float()).abs().max().item() \
            if om in ("seq_fp32", "seqsplit", "seqsplit_bf16", "conc") else 0.0
        print(json.dumps({"mode": mode, "us": round(statistics.median(res), 1), "S": S, "prefix_items": npre,
                          "decode_items": int(ditems.shape[0]), "err_vs_seq": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
