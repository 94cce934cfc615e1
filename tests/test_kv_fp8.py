"""fp8 (OCP e4m3) KV cache: layout / quantization reference on CPU, HIP kernels against the fp32 reference on the
GPU, and engine-level greedy agreement with the bf16 dense oracle (SURVEY.md §2.6 "fp8 KV").

Tolerances:
  * quantization: every element within 1/16 of its magnitude (e4m3 keeps 3 mantissa bits; the per-(token, head)
    power-of-two scale keeps every vector in the normal range) plus 2^-9 of the vector's amax (subnormals);
  * kernels: the same bound as the bf16 kernels (0.02 abs on unit-variance data), because kernel and reference read
    the SAME fp8 bytes — dequantized e4m3 * 2^e is exact in bf16, so only the accumulation order differs;
  * engine: every greedy token is within 0.15 (CPU) / 0.25 (GPU, bf16 GEMMs on top) logits of the bf16 dense
    oracle's best token. Measured on CPU, tiny-llama, 36 tokens: max gap 0.0 for fp8 as for bf16 (logit std 0.45).
"""
import math

import pytest
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import reference as ref


def _rand_kv(n, hkv, D=128, seed=0, device="cpu"):
    """Natural-order K, V [n, Hkv, 16, D] with per-(key, head) magnitudes spread over 2^-6 .. 2^1."""
    g = torch.Generator().manual_seed(seed)
    mag = lambda: torch.exp2(torch.randint(-6, 2, (n, hkv, 16, 1), generator=g).float())
    k = torch.randn(n, hkv, 16, D, generator=g) * mag()
    v = torch.randn(n, hkv, 16, D, generator=g) * mag()
    return k.to(device), v.to(device)


def _within_fp8(deq, x):
    amax = x.abs().amax(-1, keepdim=True)
    bad = (deq - x).abs() > x.abs() / 16 + amax * 2.0 ** -9 + 1e-12
    assert not bad.any(), f"{int(bad.sum())} elements outside the e4m3 bound"


def test_fp8_pack_roundtrip():
    k, v = _rand_kv(6, 2)
    kp, vp = ref.fp8_pack_pages(k, v)
    assert kp.shape == (6, 2, 16 * 128 + 32) and vp.shape == (6, 2, 128 * 16)
    k2, v2 = ref.fp8_dequant_pages(kp, vp)
    _within_fp8(k2, k)
    _within_fp8(v2.transpose(2, 3), v)


def test_cache_shapes_and_page_bytes():
    ks, vs, dt = ops.kv_cache_shapes(10, 8, 128, "fp8")
    assert dt == torch.uint8 and ks == (10, 8, 2080) and vs == (10, 8, 2048)
    assert ops.kv_page_bytes(8, 128, "fp8") * 2 < ops.kv_page_bytes(8, 128, "bf16") * 1.02
    with pytest.raises(ValueError):
        ops.kv_cache_shapes(1, 1, 128, "int4")


def test_rope_kv_write_fp8_reference_matches_bf16():
    """The fp8 writer stores the same rotated K / V as the bf16 writer, within the e4m3 bound."""
    torch.manual_seed(1)
    Hq, Hkv, D, T, nb = 8, 2, 128, 37, 5
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D).to(torch.bfloat16)
    pos = torch.randint(0, 3000, (T,))
    cs = ref.rope_cos_sin(4096, D, 500000.0)
    slots = torch.randperm(nb * 16)[:T]
    caches = {}
    for kd in ("bf16", "fp8"):
        ks, vs, dt = ops.kv_cache_shapes(nb, Hkv, D, kd)
        kc, vc = torch.zeros(ks, dtype=dt), torch.zeros(vs, dtype=dt)
        q = torch.empty(T, Hq, D, dtype=torch.bfloat16)
        ops.rope_kv_write(qkv, pos, cs, q, kc, vc, slots, Hq, Hkv)
        caches[kd] = (q, ref.gather_kv(kc, vc, torch.arange(nb), nb * 16))
    assert torch.equal(caches["bf16"][0], caches["fp8"][0])
    (kb, vb), (kf, vf) = caches["bf16"][1], caches["fp8"][1]
    _within_fp8(kf, kb)
    _within_fp8(vf, vb)


def test_engine_fp8_greedy_agreement_cpu():
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.models.oracle import dense_logits

    eng = LLMEngine(EngineConfig(model="tiny-llama", device="cpu", num_kv_blocks=256, max_model_len=2048,
                                 kv_dtype="fp8"))
    assert eng.k_cache.dtype == torch.uint8
    g = torch.Generator().manual_seed(3)
    pre = torch.randint(0, 5000, (70,), generator=g).tolist()
    prompts = [pre + torch.randint(0, 5000, (n,), generator=g).tolist() for n in (5, 17, 40)]
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    outs = eng.generate(prompts, sp)
    outs2 = eng.generate(prompts, sp)  # prefix-cached rerun reads the same fp8 pages
    assert outs == outs2
    for p, o in zip(prompts, outs):
        lg = dense_logits(eng.model, p + o)
        for i, tok in enumerate(o):
            row = lg[len(p) - 1 + i]
            assert (row.max() - row[tok]).item() < 0.15, f"token {i}: gap {(row.max() - row[tok]).item():.3f}"


# ---------------------------------------------------------------------------------------------------------------- GPU
def _close(a, b, atol, msg="", rtol=0.01):
    """|a - b| <= atol + rtol * max|b| (the rtol term covers bf16 rounding of outputs of magnitude > 1)"""
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{msg}: max err {err} > {tol}"


@pytest.mark.gpu
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8)])
@pytest.mark.parametrize("slab", [False, True])
def test_rope_kv_write_fp8_kernel(cuda, Hq, Hkv, slab):
    torch.manual_seed(2)
    D, T, nb = 128, 40, 16
    scale_rows = torch.exp2(torch.randint(-5, 4, (T, 1)).float())
    x = (torch.randn(T, (Hq + 2 * Hkv) * D) * scale_rows).to(cuda)
    qkv = torch.stack([x * 0.25, x * 0.75]) if slab else x.to(torch.bfloat16)  # slab: 2 fp32 split-K parts
    pos = torch.randint(0, 4000, (T,), device=cuda)
    cs = ref.rope_cos_sin(8192, D, 500000.0, device=cuda)
    slots = torch.randperm(nb * 16, device=cuda)[:T].long()
    slots[3] = -1
    ks, vs, dt = ops.kv_cache_shapes(nb, Hkv, D, "fp8")
    kc, vc = torch.zeros(ks, dtype=dt, device=cuda), torch.zeros(vs, dtype=dt, device=cuda)
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.rope_kv_write(qkv, pos, cs, q, kc, vc, slots, Hq, Hkv)
    kc2, vc2 = torch.zeros(ks, dtype=dt), torch.zeros(vs, dtype=dt)
    q2 = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    src = qkv.sum(0) if slab else qkv
    ref.rope_kv_write(src.cpu(), pos.cpu(), cs.cpu(), q2, kc2, vc2, slots.cpu(), Hq, Hkv)
    _close(q, q2, 0.03 * float(scale_rows.max()), "q")
    kc, vc = kc.cpu(), vc.cpu()
    # exponents identical; data bytes identical up to rare RNE ties of last-ulp-different fp32 RoPE values
    assert torch.equal(kc[..., 2048:], kc2[..., 2048:]), "exponents"
    assert (kc[..., :2048] != kc2[..., :2048]).float().mean().item() < 2e-3, "K bytes"
    assert torch.equal(vc, vc2) if not slab else (vc != vc2).float().mean().item() < 2e-3, "V bytes"
    bt = torch.arange(nb)
    (k_g, v_g), (k_r, v_r) = ref.gather_kv(kc, vc, bt, nb * 16), ref.gather_kv(kc2, vc2, bt, nb * 16)
    assert (k_g - k_r).abs().max() <= k_r.abs().max() / 8


def _fp8_paged(lens, Hkv, device, seed=0, extra=4):
    """Random fp8 pages + block tables for sequences of ``lens`` tokens (pages shuffled)."""
    B = len(lens)
    g = torch.Generator().manual_seed(seed)
    nb_total = sum((l + 15) // 16 for l in lens) + extra
    perm = torch.randperm(nb_total, generator=g)
    bt = torch.zeros(B, max((l + 15) // 16 for l in lens) + 2, dtype=torch.int32)
    c = 0
    for b, l in enumerate(lens):
        n = (l + 15) // 16
        bt[b, :n] = perm[c:c + n].int()
        c += n
    k, v = _rand_kv(nb_total, Hkv, seed=seed + 1)
    kp, vp = ref.fp8_pack_pages(k, v)
    return kp.to(device), vp.to(device), bt.to(device)


@pytest.mark.gpu
@pytest.mark.parametrize("Hq,Hkv,lens,S", [
    (32, 8, [1, 17, 300, 2049], 4),
    (8, 1, [33, 1000], 2),
    (32, 8, [5, 64, 4096], 1),
])
def test_attn_decode_fp8(cuda, Hq, Hkv, lens, S):
    torch.manual_seed(3)
    B, D = len(lens), 128
    k, v, bt = _fp8_paged(lens, Hkv, cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    o_ref, l_ref = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    part = torch.empty(B, Hq, S, D, device=cuda)
    lse = torch.empty(B, Hq, S, device=cuda)
    ops.attn_decode(q, k, v, bt, sl, None, part, lse, S, 0, scale)
    out = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    lse_o = torch.empty(B, Hq, device=cuda)
    ops.attn_merge(part, lse, out, lse_o)
    _close(out, o_ref, 0.02, "decode out")
    _close(lse_o, l_ref, 0.02, "decode lse")
    for it in range(2):  # fused merge (ticket path when S > 1)
        out2 = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode(q, k, v, bt, sl, None, part, lse, S, 0, scale, out=out2)
        _close(out2, o_ref, 0.02, f"fused decode launch {it}")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_attn_cascade_fp8(cuda, variant):
    """Shared-prefix pass on the tile kernel (fp8 LDS staging) + suffix decode (fp8 register path) == dense."""
    torch.manual_seed(4)
    Hq, Hkv, D = 32, 8, 128
    P, suffix = 160, [3, 40, 257]
    B = len(suffix)
    lens = [P + s for s in suffix]
    n_pref = P // 16
    nb_total = n_pref + sum((s + 15) // 16 + 1 for s in suffix) + 2
    kn, vn = _rand_kv(nb_total, Hkv, seed=5)
    kp, vp = ref.fp8_pack_pages(kn, vn)
    k, v = kp.to(cuda), vp.to(cuda)
    bt = torch.zeros(B, 64, dtype=torch.int32)
    c = n_pref
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        n = (lens[b] + 15) // 16 - n_pref
        bt[b, n_pref:n_pref + n] = torch.arange(c, c + n)
        c += n
    bt = bt.to(cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    ks = torch.full((B,), P, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    part = torch.empty(B, Hq, 5, D, device=cuda)
    lse = torch.empty(B, Hq, 5, device=cuda)
    items = torch.tensor([[0, B, 0, 0, 96, 0, 0, 0], [0, B, 0, 96, P, 1, 0, 0]], dtype=torch.int32, device=cuda)
    q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=cuda)
    ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out_part=part, lse_part=lse, variant=variant)
    out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
    ops.attn_decode(q, k, v, bt, sl, ks, part, lse, 3, 2, scale, out=out)
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    _close(out, o_ref, 0.02, "fp8 cascade")


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])
def test_attn_prefill_causal_fp8(cuda, Hq, Hkv, variant):
    torch.manual_seed(6)
    D = 128
    G = Hq // Hkv
    ctx, qlen = [0, 37, 512], [70, 1, 33]
    B = len(ctx)
    lens = [c + n for c, n in zip(ctx, qlen)]
    k, v, bt = _fp8_paged(lens, Hkv, cuda, seed=7)
    T = sum(qlen)
    q = torch.randn(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    q_limit = torch.empty(T, dtype=torch.int32)
    items, tile, t0 = [], ops.tile_rows(variant) // G, 0
    for b in range(B):
        for i in range(qlen[b]):
            q_limit[t0 + i] = ctx[b] + i
        for s in range(0, qlen[b], tile):
            items.append([t0 + s, min(tile, qlen[b] - s), b, 0, lens[b], -1, 0, 0])
        t0 += qlen[b]
    items = torch.tensor(items, dtype=torch.int32, device=cuda)
    q_limit = q_limit.to(cuda)
    out = torch.zeros(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out=out, variant=variant)
    out_ref = torch.zeros(T, Hq, D, dtype=torch.bfloat16)
    ref.attn_prefill_items(items.cpu(), q.cpu(), k.cpu(), v.cpu(), bt.cpu(), q_limit.cpu(), scale, out=out_ref)
    _close(out, out_ref, 0.02, "fp8 prefill")


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True], ids=["eager", "graphs"])
def test_engine_fp8_gpu_greedy_agreement(cuda, graphs):
    from kafka_llm_service_amd.engine.engine import EngineConfig, LLMEngine
    from kafka_llm_service_amd.engine.sequence import SamplingParams
    from kafka_llm_service_amd.models.oracle import dense_logits

    eng = LLMEngine(EngineConfig(model="small-llama", device=str(cuda), num_kv_blocks=1024, max_model_len=4096,
                                 kv_dtype="fp8", use_graphs=graphs))
    g = torch.Generator().manual_seed(11)
    pre = torch.randint(0, 5000, (600,), generator=g).tolist()  # long enough for the cascade pass
    prompts = [pre + torch.randint(0, 5000, (n,), generator=g).tolist() for n in (3, 60, 150, 7)]
    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    outs = eng.generate(prompts, sp)
    for p, o in zip(prompts, outs):
        lg = dense_logits(eng.model, p + o)
        for i, tok in enumerate(o):
            row = lg[len(p) - 1 + i]
            assert (row.max() - row[tok]).item() < 0.25, f"token {i}: gap {(row.max() - row[tok]).item():.3f}"
