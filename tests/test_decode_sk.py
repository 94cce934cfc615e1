"""Stream-K decode attention (ops.decode_sk_plan / attn_decode_sk, csrc/attention.hip attn_decode_sk_kernel).

CPU: the plan covers every (row, kv head) unit's key range exactly once, in pieces numbered 0..nsplit-1, within the
fused merge's 64 partial slots; the stream-K reference equals the work-item reference. GPU: the kernel against the
fp32 full-context reference, with and without cascade prefix partials, three launches back to back (the ticket
counters re-arm), and with an odd grid (empty slices)."""
import math
import random

import numpy as np
import pytest
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import reference as ref


@pytest.mark.parametrize("seed", range(6))
def test_sk_plan_covers_units(seed):
    rng = random.Random(seed)
    for _ in range(40):
        B = rng.randint(1, 70)
        hkv = rng.choice([1, 2, 8])
        P = rng.choice([0, 16, 160, 18000])
        lens = np.array([P + rng.randint(1, 3000) for _ in range(B)])
        ks = np.full(B, P)
        npre = np.full(B, 0 if P == 0 else rng.choice([0, 3, 32]))
        nwg, F = rng.choice([1, 7, 64, 512]), rng.choice([0, 1, 4, 8])
        rows, start, s_total = ops.decode_sk_plan(lens, ks, npre, hkv, nwg=nwg, F=F)
        assert rows.shape == (B + 1, 4) and start.shape == (nwg, 2) and s_total <= 64
        T, _, total = rows[B, :3]
        assert nwg * T >= total
        cov: dict = {}
        for b, h, lo, hi, sp, ns, npr in ops.decode_sk_items(rows, start, hkv):
            assert 0 <= sp < ns and npr + ns <= s_total and lo < hi
            cov.setdefault((b, h), []).append((lo, hi, sp, ns))
        assert len(cov) == B * hkv
        for (b, h), ps in cov.items():
            ps.sort()
            assert ps[0][0] == ks[b] and ps[-1][1] == lens[b]
            assert all(x[1] == y[0] for x, y in zip(ps, ps[1:]))
            assert sorted(p[2] for p in ps) == list(range(len(ps))) and all(p[3] == len(ps) for p in ps)


def _paged_with_prefix(P, suffix, Hkv, D=128, seed=7, device="cpu"):
    B = len(suffix)
    lens = [P + s for s in suffix]
    n_pref = P // 16
    nb_total = n_pref + sum((s + 15) // 16 + 1 for s in suffix) + 2
    g = torch.Generator().manual_seed(seed)
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16)
    bt = torch.zeros(B, max(lens) // 16 + 4, dtype=torch.int32)
    c = n_pref
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        n = (lens[b] + 15) // 16 - n_pref
        bt[b, n_pref:n_pref + n] = torch.arange(c, c + n)
        c += n
    return k.to(device), v.to(device), bt.to(device), lens


def test_sk_reference_matches_items_cpu():
    torch.manual_seed(0)
    Hq, Hkv, D, P = 8, 2, 128, 64
    k, v, bt, lens = _paged_with_prefix(P, [1, 40, 300, 77, 1000], Hkv)
    B = len(lens)
    q = torch.randn(B, Hq, D).to(torch.bfloat16)
    scale = 1 / math.sqrt(D)
    lens_np = np.array(lens)
    o_ref, _ = ref.attn_decode_full(q, k, v, bt, torch.tensor(lens, dtype=torch.int32), scale)
    rows, start, st = ops.decode_sk_plan(lens_np, np.zeros(B, dtype=np.int64), np.zeros(B, dtype=np.int64), Hkv,
                                         nwg=16, F=2)
    part = torch.zeros(B, Hq, st, D)
    lse = torch.full((B, Hq, st), float("-inf"))
    out = torch.empty(B, Hq, D, dtype=torch.bfloat16)
    ops.attn_decode_sk(q, k, v, bt, torch.from_numpy(rows), torch.from_numpy(start), part, lse, scale, out=out)
    assert (out.float() - o_ref.float()).abs().max().item() < 0.02


@pytest.mark.gpu
@pytest.mark.parametrize("n_pre,nwg,F", [(0, 512, 4), (3, 512, 4), (32, 512, 4), (3, 37, 0), (32, 1024, 8),
                                          (0, 3, 2)])
def test_attn_decode_sk_gpu(cuda, n_pre, nwg, F):
    torch.manual_seed(6)
    Hq, Hkv, D = 32, 8, 128
    P = 16 * 40
    suffix = [1, 29, 300, 64, 2500, 700, 33, 1200]
    k, v, bt, lens = _paged_with_prefix(P, suffix, Hkv, device=cuda)
    B = len(lens)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    lens_np = np.array(lens)
    ks = np.full(B, P if n_pre else 0)
    rows, start, st = ops.decode_sk_plan(lens_np, ks, np.full(B, n_pre), Hkv, nwg=nwg, F=F)
    part = torch.empty(B, Hq, st, D, device=cuda)
    lse = torch.empty(B, Hq, st, device=cuda)
    pre = None
    if n_pre:
        bounds = [round(P * i / n_pre / 32) * 32 for i in range(n_pre)] + [P]
        items = torch.tensor([[0, B, 0, bounds[i], bounds[i + 1], i, 0, 0] for i in range(n_pre)],
                             dtype=torch.int32, device=cuda)
        q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=cuda)
        pre = torch.empty(B, Hq, st, D, device=cuda, dtype=torch.bfloat16)
        ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out_part=pre, lse_part=lse, variant=3)
    rows_d, start_d = torch.from_numpy(rows).to(cuda), torch.from_numpy(start).to(cuda)
    for it in range(3):
        out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode_sk(q, k, v, bt, rows_d, start_d, part, lse, scale, out=out, pre_part=pre)
        _err = (out.float().cpu() - o_ref.float()).abs().max().item()
        assert _err < 0.02, f"stream-K decode n_pre={n_pre} nwg={nwg} F={F} launch {it}: max err {_err}"
