#!/usr/bin/env python3
"""Cascade tile ‖ suffix decode on disjoint CU partitions (CU-masked streams) vs the engine's sequential pair.

The cascade prefix pass (MFMA-bound, ~2 TB/s of HBM) and the suffix decode (HBM-bound, MFMA idle) of one layer are
independent except for the final log-sum-exp merge. Sequentially they cost t_tile + t_dec on the whole chip; on
two CU partitions side by side they cost ~max(t_tile(n_t CUs), t_dec(256 - n_t CUs)) + a merge. Bench shapes
(Llama-3-8B heads, 64 rows, 18k shared prefix, bench.py's suffix-length law). One JSON line per case."""
from __future__ import annotations

import argparse
import json
import random
import statistics

import numpy as np
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.engine.model_runner import decode_items


def timeit(fn, iters=20, rounds=7):
    res = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1e3 / iters)
    return statistics.median(res)


def cu_mask(a: int, n_cu: int = 256) -> list[int]:
    """a/8 of the CUs, spread evenly over the XCDs whether mask bits map to CUs XCD-major or round-robin."""
    bits = [((i % 8) + (i // 8)) % 8 < a for i in range(n_cu)]
    return [sum(1 << j for j in range(32) if bits[32 * w + j]) for w in range(n_cu // 32)]


def suffix_lengths(B: int, rng: random.Random) -> list[int]:
    out = []
    for _ in range(B):
        turn = rng.randrange(9)
        n = sum(rng.randint(32, 96) + rng.randint(128, 384) for _ in range(turn))
        out.append(n + rng.randint(32, 96) + rng.randrange(384))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=64)
    ap.add_argument("--prefix", type=int, default=18000)
    ap.add_argument("--splits", default="2,3,4")
    ap.add_argument("--probe", action="store_true", help="time the cascade tile on CU-masked streams of known masks")
    ap.add_argument("--decode-study", action="store_true", help="decode kernel alone: merge / items / length law")
    ap.add_argument("--sk-study", action="store_true", help="stream-K decode: partials only, F sweep, uniform rows")
    ap.add_argument("--seq-only", action="store_true", help="only the engine's sequential cascade + decode pair")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Hq, Hkv, D, G = 32, 8, 128, 4
    B, P = args.B, args.prefix
    torch.manual_seed(0)
    rng = random.Random(0)
    suf = suffix_lengths(B, rng)
    n_pref = P // 16
    pages = [(s + 16) // 16 + 1 for s in suf]
    nb = n_pref + sum(pages) + 16
    k = torch.randn(nb, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(nb, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
    maxb = n_pref + max(pages) + 2
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    c = n_pref
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        bt[b, n_pref:n_pref + pages[b]] = torch.arange(c, c + pages[b])
        c += pages[b]
    bt = bt.to(dev)
    lens_np = np.array([P + s for s in suf], dtype=np.int64)
    lens = torch.tensor(lens_np, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    q_limit = (lens - 1).to(torch.int32)
    scale = D ** -0.5
    out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
    suffix_bytes = sum(suf) * Hkv * D * 4

    def cascade_items(n_chunks):
        ck = -(-P // (n_chunks * 32)) * 32
        nc = -(-P // ck)
        return torch.tensor([(0, B, 0, i * ck, min(P, (i + 1) * ck), i, 0, 0) for i in range(nc)],
                            dtype=torch.int32, device=dev), nc

    def dec_items(npre, target):
        it = decode_items(lens_np, np.full(B, P, dtype=np.int64), np.full(B, npre, dtype=np.int64), Hkv,
                          target=target)
        s_total = int((npre + it[:, 4]).max())
        return torch.tensor(it, dtype=torch.int32, device=dev), s_total

    # ---- the engine today: 32 cascade chunks (bf16 partials) then the decode kernel's fused merge, whole chip
    pit, nc = cascade_items(32)
    dit, s_total = dec_items(nc, 768)
    part = torch.empty(B, Hq, s_total, D, device=dev)
    pre = torch.empty(B, Hq, s_total, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, Hq, s_total, device=dev)

    def seq():
        ops.attn_prefill(pit, q, k, v, bt, q_limit, scale, out_part=pre, lse_part=lse, variant=3)
        ops.attn_decode_items(q, k, v, bt, dit, part, lse, scale, out=out, pre_part=pre)
    t_seq = timeit(seq)
    t_tile = timeit(lambda: ops.attn_prefill(pit, q, k, v, bt, q_limit, scale, out_part=pre, lse_part=lse, variant=3))
    ref_out = out.clone()
    print(json.dumps({"case": "sequential", "cascade_chunks": nc, "decode_items": int(dit.shape[0]),
                      "us": round(t_seq, 1), "tile_us": round(t_tile, 1), "decode_us": round(t_seq - t_tile, 1),
                      "suffix_MB": round(suffix_bytes / 1e6, 1), "mean_suffix": round(sum(suf) / B)}), flush=True)
    if args.seq_only:
        return

    if args.sk_study:
        u = sum(suf) // B // 32 * 32
        for law, L in (("realistic", lens_np), ("uniform", np.full(B, P + u, dtype=np.int64))):
            it = decode_items(L, np.full(B, P, dtype=np.int64), np.zeros(B, dtype=np.int64), Hkv, target=0)
            st_i = int(it[:, 4].max())
            dit2 = torch.tensor(it, dtype=torch.int32, device=dev)
            part2 = torch.empty(B, Hq, max(st_i, 8), D, device=dev)
            lse2 = torch.empty(B, Hq, max(st_i, 8), device=dev)
            t_i = timeit(lambda: ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale))
            print(json.dumps({"case": "sk_study", "law": law, "mode": "items_target0", "us": round(t_i, 1)}),
                  flush=True)
            for nwg in (512,):
                for F in (0, 4, 16, 64):
                    rows, start, sts = ops.decode_sk_plan(L, np.full(B, P), np.zeros(B, dtype=np.int64), Hkv,
                                                          nwg=nwg, F=F)
                    rows_d = torch.from_numpy(rows).to(dev)
                    start_d = torch.from_numpy(start).to(dev)
                    part3 = torch.empty(B, Hq, sts, D, device=dev)
                    lse3 = torch.empty(B, Hq, sts, device=dev)
                    o3 = torch.empty_like(out)
                    t_p = timeit(lambda: ops.attn_decode_sk(q, k, v, bt, rows_d, start_d, part3, lse3, scale))
                    t_f = timeit(lambda: ops.attn_decode_sk(q, k, v, bt, rows_d, start_d, part3, lse3, scale,
                                                            out=o3))
                    npieces = len(ops.decode_sk_items(rows, start, Hkv))
                    print(json.dumps({"case": "sk_study", "law": law, "nwg": nwg, "F": F, "T": int(rows[-1, 0]),
                                      "pieces": npieces, "partials_us": round(t_p, 1), "fused_us": round(t_f, 1)}),
                          flush=True)
        return

    if args.decode_study:
        for npre in (32, 0):
            for target in (0, 512, 768, 1024, 1536):
                dit2, st2 = dec_items(npre, target)
                part2 = torch.empty(B, Hq, max(st2, npre + 1), D, device=dev)
                pre2 = torch.zeros(B, Hq, max(st2, npre + 1), D, device=dev, dtype=torch.bfloat16)
                lse2 = torch.full((B, Hq, max(st2, npre + 1)), -30.0, device=dev)
                t_f = timeit(lambda: ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale, out=out,
                                                            pre_part=pre2 if npre else None))
                t_p = timeit(lambda: ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale))
                print(json.dumps({"case": "decode_study", "npre": npre, "target": target,
                                  "items": int(dit2.shape[0]), "fused_us": round(t_f, 1), "partials_us": round(t_p, 1),
                                  "fused_TB/s": round(suffix_bytes / t_f / 1e6, 2),
                                  "partials_TB/s": round(suffix_bytes / t_p / 1e6, 2)}), flush=True)
        # stream-K plans (ops.decode_sk_plan): every workgroup the same cost, fused merge with 32 bf16 prefix partials
        dit2, st2 = dec_items(32, 768)
        part2 = torch.empty(B, Hq, st2, D, device=dev)
        pre2 = torch.randn(B, Hq, 64, D, device=dev).to(torch.bfloat16)
        lse_pre = torch.randn(B, Hq, 32, device=dev) - 3.0
        lse2 = torch.full((B, Hq, st2), -30.0, device=dev)
        lse2[:, :, :32] = lse_pre
        ref = torch.empty_like(out)
        ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale, out=ref, pre_part=pre2[:, :, :st2].contiguous())
        for nwg in (256, 512, 768, 1024):
            for F in (0, 2, 4, 8):
                rows, start, sts = ops.decode_sk_plan(lens_np, np.full(B, P), np.full(B, 32), Hkv, nwg=nwg, F=F)
                rows_d = torch.from_numpy(rows).to(dev)
                start_d = torch.from_numpy(start).to(dev)
                part3 = torch.empty(B, Hq, sts, D, device=dev)
                lse3 = torch.full((B, Hq, sts), -30.0, device=dev)
                lse3[:, :, :32] = lse_pre
                pre3 = pre2[:, :, :sts].contiguous()
                o3 = torch.empty_like(out)
                t_f = timeit(lambda: ops.attn_decode_sk(q, k, v, bt, rows_d, start_d, part3, lse3, scale, out=o3,
                                                        pre_part=pre3))
                err = (o3.float() - ref.float()).abs().max().item()
                print(json.dumps({"case": "decode_sk", "nwg": nwg, "F": F, "T": int(rows[-1, 0]), "s_total": sts,
                                  "fused_us": round(t_f, 1), "TB/s": round(suffix_bytes / t_f / 1e6, 2),
                                  "max_err_vs_items": round(err, 5)}), flush=True)
        # the same total suffix, uniform over the rows
        u = sum(suf) // B // 32 * 32
        lu = np.full(B, P + u, dtype=np.int64)
        for target in (0, 768):
            it = decode_items(lu, np.full(B, P, dtype=np.int64), np.zeros(B, dtype=np.int64), Hkv, target=target)
            st2 = int(it[:, 4].max())
            dit2 = torch.tensor(it, dtype=torch.int32, device=dev)
            part2 = torch.empty(B, Hq, st2, D, device=dev)
            lse2 = torch.empty(B, Hq, st2, device=dev)
            t_p = timeit(lambda: ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale))
            print(json.dumps({"case": "decode_uniform", "suffix": u, "target": target, "items": int(dit2.shape[0]),
                              "partials_us": round(t_p, 1),
                              "TB/s": round(B * u * Hkv * D * 4 / t_p / 1e6, 2)}), flush=True)
        return

    if args.probe:  # effective CU count of a mask ~ 256 x t(all) / t(mask) for this CU-bound 256-workgroup launch
        full = 0xffffffff
        masks = {"all": [full] * 8, "words0-3": [full] * 4 + [0] * 4, "words4-7": [0] * 4 + [full] * 4,
                 "even_bits": [0x55555555] * 8, "odd_bits": [0xaaaaaaaa] * 8,
                 "low16_of_each_word": [0xffff] * 8, "high16_of_each_word": [0xffff0000] * 8,
                 "bytes0_of_words": [0xff] * 8, "diag3": cu_mask(3), "diag3_complement": [(~w) & full for w in cu_mask(3)],
                 "diag4": cu_mask(4), "diag4_complement": [(~w) & full for w in cu_mask(4)], "word0": [full] + [0] * 7,
                 "words0-7_x10": [full] * 10}
        for name, m in masks.items():
            st = torch.cuda.ExternalStream(ops.ext().cu_mask_stream(m), device=dev)
            got = ops.ext().stream_cu_mask(st.cuda_stream, 10)
            ev0, ev1 = torch.cuda.Event(), torch.cuda.Event()

            def f():
                ev0.record(torch.cuda.current_stream())
                st.wait_event(ev0)
                with torch.cuda.stream(st):
                    ops.attn_prefill(pit, q, k, v, bt, q_limit, scale, out_part=pre, lse_part=lse, variant=3)
                    ev1.record(st)
                torch.cuda.current_stream().wait_event(ev1)
            t = timeit(f)
            print(json.dumps({"case": "probe", "mask": name, "bits": sum(bin(x).count("1") for x in m[:8]),
                              "readback": [hex(x) for x in got], "tile_us": round(t, 1),
                              "eff_cus": round(256 * t_tile / t)}), flush=True)
        return

    # ---- partitions: a/8 of the CUs for the cascade, the rest for the decode; merge on the whole chip
    main_s = torch.cuda.current_stream()
    ev0, ev_a, ev_b = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()
    for a in [int(x) for x in args.splits.split(",")]:
        n_t = 32 * a
        sa = torch.cuda.ExternalStream(ops.ext().cu_mask_stream(cu_mask(a)), device=dev)
        sb = torch.cuda.ExternalStream(ops.ext().cu_mask_stream([(~w) & 0xffffffff for w in cu_mask(a)]),
                                       device=dev)
        for chunks in sorted({n_t // Hkv, 2 * n_t // Hkv, 32}):
            chunks = min(chunks, 48)
            pit2, nc2 = cascade_items(chunks)
            for target in (2 * (256 - n_t), 3 * (256 - n_t), 768):
                dit2, st2 = dec_items(nc2, target)
                part2 = torch.empty(B, Hq, st2, D, device=dev)
                lse2 = torch.empty(B, Hq, st2, device=dev)

                def tile_only():
                    with torch.cuda.stream(sa):
                        ops.attn_prefill(pit2, q, k, v, bt, q_limit, scale, out_part=part2, lse_part=lse2, variant=3)

                def dec_only():
                    with torch.cuda.stream(sb):
                        ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale)

                def par(merge=True):
                    ev0.record(main_s)
                    sa.wait_event(ev0)
                    sb.wait_event(ev0)
                    with torch.cuda.stream(sa):
                        ops.attn_prefill(pit2, q, k, v, bt, q_limit, scale, out_part=part2, lse_part=lse2, variant=3)
                        ev_a.record(sa)
                    with torch.cuda.stream(sb):
                        ops.attn_decode_items(q, k, v, bt, dit2, part2, lse2, scale)
                        ev_b.record(sb)
                    main_s.wait_event(ev_a)
                    main_s.wait_event(ev_b)
                    if merge:
                        ops.attn_merge(part2, lse2, out)

                def timed_on(stream_fn, s):
                    # time a side-stream launch from the main stream's clock (join before the end event)
                    def f():
                        ev0.record(main_s)
                        s.wait_event(ev0)
                        stream_fn()
                        ev_a.record(s)
                        main_s.wait_event(ev_a)
                    return timeit(f)
                t_a = timed_on(tile_only, sa)
                t_b = timed_on(dec_only, sb)
                t_par = timeit(lambda: par(False))
                t_parm = timeit(par)
                par()
                torch.cuda.synchronize()
                err = (out.float() - ref_out.float()).abs().max().item()
                print(json.dumps({"case": "partition", "tile_cus": n_t, "cascade_chunks": nc2, "decode_target": target,
                                  "decode_items": int(dit2.shape[0]), "tile_us": round(t_a, 1),
                                  "decode_us": round(t_b, 1), "par_us": round(t_par, 1),
                                  "par_merge_us": round(t_parm, 1), "vs_seq": round(t_seq / t_parm, 3),
                                  "max_err": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
