"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference of the same op (ops/reference.py)."""
import math

import pytest
import torch

from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"{msg} max err {err} > {tol}"


@pytest.mark.parametrize("T,d", [(1, 4096), (64, 4096), (37, 8192), (5, 1024), (3, 4104)])
def test_rmsnorm(cuda, T, d):
    torch.manual_seed(0)
    x = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(d, device=cuda, dtype=torch.bfloat16)
    y = ops.rmsnorm(x, w, 1e-5)
    _close(y, ref.rmsnorm(x.cpu(), w.cpu(), 1e-5), atol=0.05, rtol=0.01, msg="rmsnorm")


@pytest.mark.parametrize("T,d", [(1, 4096), (64, 4096), (130, 8192)])
def test_fused_add_rmsnorm(cuda, T, d):
    torch.manual_seed(1)
    x = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    r = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    w = torch.randn(d, device=cuda, dtype=torch.bfloat16)
    y_ref, s_ref = ref.fused_add_rmsnorm(x.cpu(), r.cpu(), w.cpu(), 1e-5)
    y = ops.fused_add_rmsnorm(x, r, w, 1e-5)
    _close(r, s_ref, atol=1e-2, msg="residual")
    _close(y, y_ref, atol=0.05, rtol=0.01, msg="norm")


@pytest.mark.parametrize("T,F", [(1, 14336), (64, 14336), (7, 1024)])
def test_silu_mul(cuda, T, F):
    x = torch.randn(T, 2 * F, device=cuda, dtype=torch.bfloat16)
    _close(ops.silu_mul(x), ref.silu_mul(x.cpu()), atol=0.03, rtol=0.01)


def _make_cache(nb, Hkv, D=128, device="cpu"):
    k = torch.zeros(nb, Hkv, 16, D, dtype=torch.bfloat16, device=device)
    v = torch.zeros(nb, Hkv, D, 16, dtype=torch.bfloat16, device=device)
    return k, v


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])
def test_rope_kv_write(cuda, Hq, Hkv):
    torch.manual_seed(2)
    D, T, nb = 128, 40, 16
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=cuda, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=cuda, dtype=torch.long)
    cs = ref.rope_cos_sin(8192, D, 500000.0, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                               "high_freq_factor": 4.0, "original_max_position_embeddings": 8192},
                          device=cuda)
    slots = torch.randperm(nb * 16, device=cuda)[:T].long()
    slots[3] = -1
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    k, v = _make_cache(nb, Hkv, D, cuda)
    ops.rope_kv_write(qkv, pos, cs, q, k, v, slots, Hq, Hkv)
    q2 = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    k2, v2 = _make_cache(nb, Hkv, D)
    ref.rope_kv_write(qkv.cpu(), pos.cpu(), cs.cpu(), q2, k2, v2, slots.cpu(), Hq, Hkv)
    _close(q, q2, atol=0.03, rtol=0.01, msg="q")
    _close(k, k2, atol=0.03, rtol=0.01, msg="k")
    assert torch.equal(v.cpu(), v2), "v cache"


def _random_paged(B, lens, Hkv, device, seed=0, D=128):
    g = torch.Generator().manual_seed(seed)
    max_nb = max((l + 15) // 16 for l in lens)
    nb_total = sum((l + 15) // 16 for l in lens) + 4
    perm = torch.randperm(nb_total, generator=g)
    bt = torch.zeros(B, max_nb + 2, dtype=torch.int32)
    c = 0
    for b, l in enumerate(lens):
        n = (l + 15) // 16
        bt[b, :n] = perm[c:c + n].int()
        c += n
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16)
    return k.to(device), v.to(device), bt.to(device)


@pytest.mark.parametrize("Hq,Hkv,lens,S", [
    (32, 8, [1, 17, 300, 2049], 4),
    (32, 8, [4096] * 3, 8),
    (8, 1, [33, 1000], 2),
    (32, 8, [5, 64], 1),
])
def test_attn_decode(cuda, Hq, Hkv, lens, S):
    torch.manual_seed(3)
    B, D = len(lens), 128
    k, v, bt = _random_paged(B, lens, Hkv, cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    part = torch.empty(B, Hq, S, D, device=cuda)
    lse = torch.empty(B, Hq, S, device=cuda)
    ops.attn_decode(q, k, v, bt, sl, None, part, lse, S, 0, scale)
    out = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    lse_o = torch.empty(B, Hq, device=cuda)
    ops.attn_merge(part, lse, out, lse_o)
    o_ref, l_ref = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    _close(out, o_ref, atol=0.02, msg="decode out")
    _close(lse_o, l_ref, atol=0.02, msg="decode lse")


@pytest.mark.parametrize("n_pre,S", [(0, 1), (1, 1), (3, 1), (6, 1), (0, 4), (3, 5), (0, 32)])
def test_attn_decode_fused_merge(cuda, n_pre, S):
    """The decode kernel merges the cascade-prefix partials itself and writes bf16 rows: directly with one split per
    sequence, through ticket counters (last split merges) with several. Three launches back to back check that the
    counters re-arm."""
    torch.manual_seed(6)
    Hq, Hkv, D = 32, 8, 128
    P = 16 * 12
    suffix = [1, 29, 300, 64]
    B = len(suffix)
    lens = [P + s for s in suffix]
    n_pref = P // 16
    nb_total = n_pref + sum((s + 15) // 16 + 1 for s in suffix) + 2
    g = torch.Generator().manual_seed(7)
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16).to(cuda)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16).to(cuda)
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
    scale = 1 / math.sqrt(D)
    part = torch.empty(B, Hq, n_pre + S, D, device=cuda)
    lse = torch.empty(B, Hq, n_pre + S, device=cuda)
    if n_pre:
        bounds = [round(P * i / n_pre / 32) * 32 for i in range(n_pre)] + [P]
        items = torch.tensor([[0, B, 0, bounds[i], bounds[i + 1], i, 0, 0] for i in range(n_pre)],
                             dtype=torch.int32, device=cuda)
        q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=cuda)
        ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out_part=part, lse_part=lse)
        ks = torch.full((B,), P, dtype=torch.int32, device=cuda)
    else:
        ks = None
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    for it in range(3):
        out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode(q, k, v, bt, sl, ks, part, lse, S, n_pre, scale, out=out)
        _close(out, o_ref, atol=0.02, msg=f"fused merge n_pre={n_pre} S={S} launch {it}")


@pytest.mark.parametrize("Hkv,G,rows,S2", [(8, 4, 105, 13), (4, 8, 3, 1), (8, 2, 9, 40), (2, 3, 5, 4)])
def test_attn_decode_merges_prefill_rows(cuda, Hkv, G, rows, S2):
    """Extra workgroups of the decode launch merge other rows' fp32 partials (attention.hip FusedMerge: a step's
    prefill rows once every prefill tile rode in the cascade launch) as attn_merge does — unwritten slots (lse -inf,
    NaN data) weigh nothing, rows outside the range stay untouched — and the decode rows are unchanged."""
    torch.manual_seed(11)
    D, Hq = 128, Hkv * G
    lens = [40, 300, 17]
    B = len(lens)
    k, v, bt = _random_paged(B, lens, Hkv, cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    items = ops.uniform_decode_items(sl, None, 1, 0)
    part = torch.empty(B, Hq, 1, D, device=cuda)
    lse = torch.empty(B, Hq, 1, device=cuda)
    mp = torch.randn(rows, Hq, S2, D, device=cuda)
    ml = torch.randn(rows, Hq, S2, device=cuda) * 4
    if S2 > 1:
        ml[:, :, -1] = float("-inf")
        mp[:, :, -1] = float("nan")
    out = torch.full((B + 1 + rows + 1, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
    ops.attn_decode_items(q, k, v, bt, items, part, lse, scale, out=out[:B], merge=(mp, ml, out[B + 1:B + 1 + rows]))
    torch.cuda.synchronize()
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    _close(out[:B], o_ref, atol=0.02, msg="decode rows")
    m_ref = torch.empty(rows, Hq, D)
    ref.attn_merge(mp.cpu(), ml.cpu(), m_ref)
    _close(out[B + 1:B + 1 + rows], m_ref, atol=0.02, msg="merged prefill rows")
    assert torch.isnan(out[B].float()).all() and torch.isnan(out[-1].float()).all(), "rows outside the merge range"


def test_attn_decode_multi_group_cascade(cuda):
    """Three prefix groups (different shared prefixes of 208 / 320 / 96 tokens) + two ungrouped rows, planned by the
    engine's own planner (model_runner.prefix_groups / decode_items, long suffixes split into pieces), run as
    prefix tile passes + the work-item decode kernel with its fused merge == dense attention per row."""
    import numpy as np

    from kafka_llm_service_amd.engine.model_runner import decode_items, prefix_groups

    torch.manual_seed(8)
    Hq, Hkv, D = 32, 8, 128
    prefixes = [208, 320, 96]
    members = [[0, 3, 5, 8], [1, 6], [2, 7, 9]]  # rows 4 and 10 stay ungrouped
    suffix = [5, 700, 33, 1900, 450, 64, 17, 1, 300, 90, 2500]
    B = len(suffix)
    g = torch.Generator().manual_seed(9)
    pages = iter(torch.randperm(4000, generator=g).tolist())
    pre_pages = [[next(pages) for _ in range(P // 16)] for P in prefixes]
    lens, rows = [], []
    for b in range(B):
        grp = [i for i, m in enumerate(members) if b in m]
        base = pre_pages[grp[0]] if grp else []
        L = len(base) * 16 + suffix[b]
        rows.append(base + [next(pages) for _ in range((L + 15) // 16 - len(base))])
        lens.append(L)
    W = max(len(r) for r in rows)
    bt_np = np.zeros((B, W), dtype=np.int32)
    for b, r in enumerate(rows):
        bt_np[b, :len(r)] = r
    order, groups = prefix_groups(bt_np, (np.array(lens) - 1) // 16, min_blocks=4)
    assert len(groups) == 3
    bt_np, lens = bt_np[order], [lens[i] for i in order]
    seq_lens = np.array(lens)
    kv_start, npre = np.zeros(B, dtype=np.int64), np.zeros(B, dtype=np.int64)
    pit, r0 = [], 0
    for n, p in groups:
        P, nc = p * 16, 3
        ck = -(-P // (nc * 32)) * 32
        nc = -(-P // ck)
        pit += [(r0, n, r0, c * ck, min(P, (c + 1) * ck), c, 0, 0) for c in range(nc)]
        kv_start[r0:r0 + n], npre[r0:r0 + n] = P, nc
        r0 += n
    dit = decode_items(seq_lens, kv_start, npre, Hkv, target=64)
    assert (dit[:, 4] > 1).any()  # some suffix is split into pieces (ticket merge)
    S_total = int((npre[dit[:, 0]] + dit[:, 4]).max())
    k = torch.randn(4000, Hkv, 16, D, generator=g).to(torch.bfloat16).to(cuda)
    v = torch.randn(4000, Hkv, D, 16, generator=g).to(torch.bfloat16).to(cuda)
    bt = torch.from_numpy(bt_np).to(cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    part = torch.empty(B, Hq, S_total, D, device=cuda)
    lse = torch.empty(B, Hq, S_total, device=cuda)
    q_limit = torch.tensor(lens, dtype=torch.int32, device=cuda) - 1
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), torch.tensor(lens), scale)
    for launch in range(2):
        ops.attn_prefill(torch.tensor(pit, dtype=torch.int32, device=cuda), q, k, v, bt, q_limit, scale,
                         out_part=part, lse_part=lse)
        out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode_items(q, k, v, bt, torch.from_numpy(dit).to(cuda), part, lse, scale, out=out)
        _close(out, o_ref, atol=0.02, msg=f"multi-group cascade launch {launch}")


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_attn_decode_kv_start_cascade(cuda, variant):
    """Cascade: prefix partial from attn_prefill (rows = decode seqs) + suffix partial from attn_decode == full."""
    torch.manual_seed(4)
    Hq, Hkv, D = 32, 8, 128
    P = 160  # shared prefix length (multiple of 16)
    suffix = [3, 40, 257]
    B = len(suffix)
    lens = [P + s for s in suffix]
    g = torch.Generator().manual_seed(5)
    n_pref = P // 16
    nb_total = n_pref + sum((s + 15) // 16 + 1 for s in suffix) + 2
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16).to(cuda)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16).to(cuda)
    bt = torch.zeros(B, 64, dtype=torch.int32)
    c = n_pref
    for b, s in enumerate(suffix):
        bt[b, :n_pref] = torch.arange(n_pref)
        n = (lens[b] + 15) // 16 - n_pref
        bt[b, n_pref:n_pref + n] = torch.arange(c, c + n)
        c += n
    bt = bt.to(cuda)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    ks = torch.full((B,), P, dtype=torch.int32, device=cuda)
    scale = 1 / math.sqrt(D)
    S_pre, S_suf = 2, 3
    S_total = S_pre + S_suf
    part = torch.empty(B, Hq, S_total, D, device=cuda)
    lse = torch.empty(B, Hq, S_total, device=cuda)
    # prefix: rows are the B decode sequences, all using block table row 0 restricted to [0, P), split in 2 chunks
    items = torch.tensor([[0, B, 0, 0, 96, 0, 0, 0], [0, B, 0, 96, P, 1, 0, 0]], dtype=torch.int32, device=cuda)
    q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=cuda)
    ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out_part=part, lse_part=lse, variant=variant)
    ops.attn_decode(q, k, v, bt, sl, ks, part, lse, S_suf, S_pre, scale)
    out = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.attn_merge(part, lse, out)
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
    _close(out, o_ref, atol=0.02, msg="cascade")


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8)])
def test_attn_prefill_causal(cuda, Hq, Hkv, variant):
    torch.manual_seed(6)
    D = 128
    G = Hq // Hkv
    ctx = [0, 37, 512]     # cached context per sequence
    qlen = [70, 1, 33]     # new tokens per sequence
    B = len(ctx)
    lens = [c + n for c, n in zip(ctx, qlen)]
    k, v, bt = _random_paged(B, lens, Hkv, cuda, seed=7)
    T = sum(qlen)
    q = torch.randn(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    q_limit = torch.empty(T, dtype=torch.int32)
    items = []
    tile = ops.tile_rows(variant) // G
    t0 = 0
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
    _close(out, out_ref, atol=0.02, msg="prefill")


@pytest.mark.parametrize("variant", [0, 3])
@pytest.mark.parametrize("spike_at", [5, 300, 1500])
def test_attn_tile_rescale_spike(cuda, variant, spike_at):
    """Forces the online-softmax rescale branch at a chosen key (cdna_hip_programming.md §5.4 rule 26): one key row
    scaled x12 makes every query's running max jump there (variant 3 rescales only past 2^8 growth, so the jump must
    be large and the O / l / pending-P scaling exact). Non-causal rows over a 2,000-key range (31 ring tiles: the
    3-slot DMA ring wraps many times), split into two key chunks with partials, vs the fp32 reference."""
    torch.manual_seed(11)
    Hq, Hkv, D, B = 32, 8, 128, 64
    L = 2000
    k, v, bt = _random_paged(1, [L], Hkv, cuda, seed=12)
    pg, off = bt[0, spike_at // 16].item(), spike_at % 16
    ref.k_planes(k)[pg, :, :, off, :] *= 12  # the whole key row (pages are stored plane-major)
    q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    G = Hq // Hkv
    tile = ops.tile_rows(variant) // G
    items = [[t0, min(tile, B - t0), 0, c0, c1, c, 0, 0] for t0 in range(0, B, tile)
             for c, (c0, c1) in enumerate([(0, 1024), (1024, L)])]
    items = torch.tensor(items, dtype=torch.int32, device=cuda)
    q_limit = torch.full((B,), L - 1, dtype=torch.int32, device=cuda)
    bt_rows = bt[:1].expand(B, -1).contiguous()
    part = torch.empty(B, Hq, 2, D, device=cuda)
    lse = torch.empty(B, Hq, 2, device=cuda)
    ops.attn_prefill(items, q, k, v, bt_rows, q_limit, 1 / math.sqrt(D), out_part=part, lse_part=lse,
                     variant=variant)
    out = torch.empty(B, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.attn_merge(part, lse, out)
    o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt_rows.cpu(), torch.full((B,), L), 1 / math.sqrt(D))
    _close(out, o_ref, atol=0.02, msg=f"spike at {spike_at}")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_sample_greedy(cuda, dtype):
    torch.manual_seed(8)
    B, V = 17, 128256
    logits = torch.randn(B, V, device=cuda).to(dtype)
    temp = torch.zeros(B, device=cuda)
    tok = ops.sample(logits, temp)
    assert torch.equal(tok.cpu(), torch.argmax(logits.float(), -1).cpu())


def test_sample_distribution(cuda):
    """Gumbel-max with temperature reproduces softmax(x/T); top-k / top-p never leave their sets."""
    V = 64
    logits = torch.randn(1, V, device=cuda) * 2
    n = 4000
    lg = logits.expand(n, V).contiguous()
    temp = torch.full((n,), 0.8, device=cuda)
    seeds = torch.arange(n, device=cuda, dtype=torch.long)
    tok = ops.sample(lg, temp, seeds=seeds).cpu()
    emp = torch.bincount(tok, minlength=V).float() / n
    p = torch.softmax(logits[0].cpu() / 0.8, -1)
    assert (emp - p).abs().max().item() < 0.05
    topk = torch.full((n,), 5, device=cuda, dtype=torch.int32)
    tok = ops.sample(lg, temp, top_k=topk, seeds=seeds).cpu()
    allowed = set(torch.topk(logits[0].cpu(), 5).indices.tolist())
    assert set(tok.tolist()) <= allowed
    topp = torch.full((n,), 0.5, device=cuda)
    tok = ops.sample(lg, temp, top_p=topp, seeds=seeds).cpu()
    ps, order = torch.sort(p, descending=True)
    keep = (torch.cumsum(ps, 0) - ps) < 0.5
    allowed = set(order[keep].tolist())
    assert set(tok.tolist()) <= allowed


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (128, 8, 2), (3000, 8, 2), (77, 16, 4), (2048, 8, 4), (5000, 8, 2)])
def test_moe_route(cuda, T, E, k):
    torch.manual_seed(7)
    logits = torch.randn(T, E, device=cuda).to(torch.bfloat16)
    r = ops.moe_route(logits, k)
    tw, te, pt, pw, eo, to = ref.moe_route(logits.cpu(), k, ops.GG_BM)
    assert torch.equal(r.topk_e.cpu(), te) and torch.equal(r.expert_off.cpu(), eo)
    assert torch.equal(r.tile_off.cpu(), to) and torch.equal(r.perm_tok.cpu(), pt)
    _close(r.topk_w, tw, atol=1e-5, msg="topk_w")
    _close(r.perm_w, pw, atol=1e-5, msg="perm_w")


@pytest.mark.parametrize("T,d,N,E,e_lo,e_n", [(128, 512, 1024, 8, 0, 8), (300, 1024, 512, 8, 2, 4),
                                              (1, 256, 384, 8, 0, 8), (64, 4096, 2048, 8, 0, 8)])
def test_grouped_gemm(cuda, T, d, N, E, e_lo, e_n):
    torch.manual_seed(8)
    x = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(e_n, N, d, device=cuda) * d ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(e_n, d, N, device=cuda) * N ** -0.5).to(torch.bfloat16)
    r = ops.moe_route(torch.randn(T, E, device=cuda).to(torch.bfloat16), 2)
    rc = ops.MoERouting(*(t.cpu() for t in (r.topk_w, r.topk_e, r.perm_tok, r.perm_w, r.expert_off, r.tile_off)),
                        E)
    # gather mode -> bf16 rows (only the local experts' segments are defined)
    y = ops.grouped_gemm(x, w, r, gather=True, e_lo=e_lo)
    y_ref = torch.zeros(T * 2, N)
    ref.grouped_gemm(x.cpu(), w.cpu(), rc.perm_tok, rc.perm_w, rc.expert_off, e_lo, True, y_ref, None)
    eo = rc.expert_off.tolist()
    a, b = eo[e_lo], eo[e_lo + e_n]
    _close(y[a:b], y_ref[a:b], atol=0.03, rtol=0.01, msg="gather")
    # direct mode with the fused weighted scatter-combine
    h = torch.randn(T * 2, N, device=cuda, dtype=torch.bfloat16)
    out = torch.zeros(T, d, device=cuda)
    ops.grouped_gemm(h, w2, r, gather=False, e_lo=e_lo, combine_out=out)
    out_ref = torch.zeros(T, d)
    ref.grouped_gemm(h.cpu(), w2.cpu(), rc.perm_tok, rc.perm_w, rc.expert_off, e_lo, False, None, out_ref)
    _close(out, out_ref, atol=0.02, rtol=0.01, msg="combine")


@pytest.mark.parametrize("T,d,F,E,e_lo,e_n", [(1, 512, 512, 8, 0, 8), (37, 1024, 768, 8, 0, 8),
                                              (64, 4096, 1792, 8, 0, 8), (128, 512, 1024, 8, 2, 4),
                                              (100, 768, 256, 8, 4, 4), (300, 1024, 512, 8, 0, 8),
                                              (640, 512, 512, 8, 0, 8), (256, 512, 1024, 8, 0, 8),
                                              (200, 512, 1024, 8, 2, 4), (400, 4096, 1792, 8, 0, 8)])
def test_wstream_grouped(cuda, T, d, F, E, e_lo, e_n):
    """Expert MLP on the grouped weight-streaming kernel (GLU-tiled w13 with fused SwiGLU, w2 with the fused weighted
    combine) vs the fp32 reference of the same routing, including an expert-parallel subset of experts."""
    torch.manual_seed(9)
    x = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    w13 = (torch.randn(e_n, 2 * F, d, device=cuda) * d ** -0.5).to(torch.bfloat16)
    w2 = (torch.randn(e_n, d, F, device=cuda) * F ** -0.5).to(torch.bfloat16)
    r = ops.moe_route(torch.randn(T, E, device=cuda).to(torch.bfloat16), 2)
    rc = ops.MoERouting(*(t.cpu() for t in (r.topk_w, r.topk_e, r.perm_tok, r.perm_w, r.expert_off, r.tile_off)),
                        E)
    w13t, w2t = ops.tile_experts(w13, glu=True), ops.tile_experts(w2)
    assert torch.equal(ops.untile_experts(w13t, glu=True), w13)
    a = ops.grouped_stream_glu(x, w13t, r, e_lo=e_lo)
    h_ref = torch.zeros(T * 2, 2 * F)
    ref.grouped_gemm(x.cpu().float(), w13.cpu().float(), rc.perm_tok, rc.perm_w, rc.expert_off, e_lo, True, h_ref,
                     None)
    eo = rc.expert_off.tolist()
    lo, hi = eo[e_lo], eo[e_lo + e_n]
    _close(a[lo:hi], ref.silu_mul(h_ref[lo:hi]), atol=0.03, rtol=0.02, msg="grouped glu")
    out = torch.zeros(T, d, device=cuda)
    ops.grouped_stream_combine(a, w2t, r, T, out, e_lo=e_lo)
    out_ref = torch.zeros(T, d)
    ref.grouped_gemm(a.cpu(), w2.cpu(), rc.perm_tok, rc.perm_w, rc.expert_off, e_lo, False, None, out_ref)
    _close(out, out_ref, atol=0.02, rtol=0.01, msg="grouped combine")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M", [1, 7, 32, 33, 64, 65, 80, 96, 97, 128, 129, 169, 192, 193, 200, 256])
@pytest.mark.parametrize("N,K", [(6144, 4096), (4096, 14336), (1280, 8192), (16032, 1024), (96, 512)])
def test_wstream_gemm(cuda, M, N, K):
    """Weight-streaming decode GEMM on wave-tiled weights (bf16 direct and split-K slabs) vs fp32 matmul."""
    torch.manual_seed(11)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    wt = ops.tile_weight(w)
    assert torch.equal(ops.untile_weight(wt), w)
    ref_y = x.float() @ w.float().t()
    for ms in (1, 8):
        y = ops.linear_stream(x, wt, max_splits=ms)
        plan = ops.stream_plan(M, N, K, ms)
        if plan[2] == 1:
            assert y.dtype == torch.bfloat16 and y.shape == (M, N)
        else:
            assert ops.is_slab(y) and y.shape == (plan[2], M, N)
        _close(ops.slab_reduce(y), ref_y, atol=0.02, rtol=0.01, msg=f"wstream M={M} N={N} K={K} ms={ms}")
        torch.cuda.synchronize()


@pytest.mark.parametrize("M", [17, 64, 128, 169])
def test_wstream_slabs_reused_buffer(cuda, M):
    """The split-K slabs leave the GEMM as sc1 stores (their lines bypass the writer XCD's L2). Rewrite ONE slab buffer
    many times after consumers on every XCD have read (and cached) its previous contents, as the engine does layer
    after layer, and check every round against fp32: no reader may see a stale line."""
    ext = ops._ext.load()
    N, K = 6144, 4096
    w = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    wt = ops.tile_weight(w)
    mt, kc, S = ops.stream_plan(M, N, K)
    assert S > 1
    p = torch.empty(S, M, N, device=cuda)
    y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    g = torch.Generator(device=cuda).manual_seed(5)
    for it in range(6):
        x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, generator=g)
        ext.wstream_gemm(x, wt, None, p, 8, True, False)
        ext.slab_reduce(p, y)                      # our kernel, every XCD
        s2 = p.sum(0)                              # a torch kernel reading the same lines
        ref_y = x.float() @ w.float().t()
        _close(y, ref_y, atol=0.02, rtol=0.01, msg=f"slab_reduce round {it}")
        _close(s2, ref_y, atol=0.02, rtol=0.01, msg=f"torch sum round {it}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M", [130, 200, 256])
def test_skinny_slabs_reused_buffer(cuda, M):
    """As test_wstream_slabs_reused_buffer for the skinny GEMM's sc1 slab stores (129..256-row steps)."""
    ext = ops._ext.load()
    N, K = 4096, 14336
    w = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    wt = ops.tile_weight(w)
    S = ops.skinny_plan(M, N, K)
    assert S > 1
    p = torch.empty(S, M, N, device=cuda)
    y = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    g = torch.Generator(device=cuda).manual_seed(6)
    for it in range(6):
        x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, generator=g)
        ext.skinny_gemm(x, wt, None, p, S, False)
        ext.slab_reduce(p, y)
        s2 = p.sum(0)
        ref_y = x.float() @ w.float().t()
        _close(y, ref_y, atol=0.03, rtol=0.01, msg=f"skinny slab_reduce round {it}")
        _close(s2, ref_y, atol=0.03, rtol=0.01, msg=f"skinny torch sum round {it}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M", [1, 40, 64, 80, 100, 150, 168, 192, 256])
@pytest.mark.parametrize("N,K", [(28672, 4096), (7168, 8192), (2048, 1024)])
def test_wstream_glu(cuda, M, N, K):
    """GLU-tiled gate_up: fused silu(gate) * up epilogue (one split) and de-interleaved gate | up slabs (split plans)
    vs the fp32 reference."""
    torch.manual_seed(13)
    x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=cuda) * 0.05).to(torch.bfloat16)
    wt = ops.tile_weight(w, glu=True)
    assert torch.equal(ops.untile_weight(wt, glu=True), w)
    y_ref = x.float() @ w.float().t()
    a = ops.linear_glu(x, wt)
    _close(a, ref.silu_mul(y_ref.cpu()), atol=0.03, rtol=0.02, msg=f"glu M={M} N={N} K={K}")
    for ms in (1, 8):
        y = ops.linear_stream(x, wt, max_splits=ms, glu=True)
        if ops.is_slab(y):
            _close(ops.slab_reduce(y), y_ref, atol=0.02, rtol=0.01, msg=f"glu slab M={M} N={N} ms={ms}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("T", [1, 37, 64])
def test_slab_consumers(cuda, T):
    """fused_add_rmsnorm / silu_mul / rope_kv_write fed with split-K slabs == the same ops on the summed input."""
    torch.manual_seed(12)
    S, d, F = 4, 4096, 2048
    p = torch.randn(S, T, d, device=cuda)
    r1 = torch.randn(T, d, device=cuda, dtype=torch.bfloat16)
    r2 = r1.clone()
    w = torch.randn(d, device=cuda, dtype=torch.bfloat16)
    y = ops.fused_add_rmsnorm(p, r1, w, 1e-5)
    y_ref, s_ref = ref.fused_add_rmsnorm(p.sum(0).cpu(), r2.cpu(), w.cpu(), 1e-5)
    _close(r1, s_ref, atol=2e-2, rtol=1e-2, msg="slab residual")
    _close(y, y_ref, atol=0.05, rtol=0.01, msg="slab norm")
    g = torch.randn(S, T, 2 * F, device=cuda)
    _close(ops.silu_mul(g), ref.silu_mul(g.sum(0).cpu()), atol=0.03, rtol=0.01, msg="slab silu")
    Hq, Hkv, D, nb = 32, 8, 128, 8
    qkv = torch.randn(S, T, (Hq + 2 * Hkv) * D, device=cuda)
    pos = torch.randint(0, 4000, (T,), device=cuda, dtype=torch.long)
    cs = ref.rope_cos_sin(8192, D, 500000.0, None, device=cuda)
    slots = torch.randperm(nb * 16, device=cuda)[:T].long()
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    k, v = _make_cache(nb, Hkv, D, cuda)
    ops.rope_kv_write(qkv, pos, cs, q, k, v, slots, Hq, Hkv)
    q2 = torch.empty(T, Hq, D, dtype=torch.bfloat16)
    k2, v2 = _make_cache(nb, Hkv, D)
    ref.rope_kv_write(qkv.sum(0).cpu(), pos.cpu(), cs.cpu(), q2, k2, v2, slots.cpu(), Hq, Hkv)
    _close(q, q2, atol=0.05, rtol=0.01, msg="slab q")
    _close(k, k2, atol=0.05, rtol=0.01, msg="slab k")
    _close(v, v2, atol=0.02, rtol=0.01, msg="slab v")


@pytest.mark.parametrize("ctx,qlen", [(0, 2048), (300, 1000)])
def test_attn_prefill_balanced_split(cuda, ctx, qlen):
    """Causal prefill planned by model_runner.plan_prefill_items: long tiles split into key pieces (partials merged
    per row range), short tiles written directly, all in one launch == the fp32 reference."""
    from kafka_llm_service_amd.engine.model_runner import plan_prefill_items

    torch.manual_seed(12)
    Hq, Hkv, D = 32, 8, 128
    G = Hq // Hkv
    L = ctx + qlen
    k, v, bt = _random_paged(1, [L], Hkv, cuda, seed=13)
    q = torch.randn(qlen, Hq, D, device=cuda, dtype=torch.bfloat16)
    q_limit = torch.arange(ctx, L, dtype=torch.int32)
    tile = ops.tile_rows(0) // G
    tiles = [(t0, min(tile, qlen - t0), 0, ctx + t0 + min(tile, qlen - t0), L) for t0 in range(0, qlen, tile)]
    items, splits, ranges = plan_prefill_items(tiles, Hkv, 256, 256)
    assert splits >= 2 and ranges
    it = torch.tensor(items, dtype=torch.int32, device=cuda)
    out = torch.full((qlen, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
    part = torch.empty(qlen, Hq, splits, D, device=cuda)
    lse = torch.full((qlen, Hq, splits), float("-inf"), device=cuda)
    scale = 1 / math.sqrt(D)
    ops.attn_prefill(it, q, k, v, bt, q_limit.to(cuda), scale, out=out, out_part=part, lse_part=lse)
    for lo, hi in ranges:
        ops.attn_merge(part[lo:hi], lse[lo:hi], out[lo:hi])
    whole = torch.tensor([[t0, cnt, 0, 0, L, -1, 0, 0] for t0, cnt, _, _, _ in tiles], dtype=torch.int32)
    out_ref = torch.zeros(qlen, Hq, D, dtype=torch.bfloat16)
    ref.attn_prefill_items(whole, q.cpu(), k.cpu(), v.cpu(), bt.cpu(), q_limit, scale, out=out_ref)
    _close(out, out_ref, atol=0.02, msg="balanced split prefill")


def test_sample_split_rows_equal_one_workgroup(cuda):
    """Greedy and plain-temperature rows split over 8 workgroups (ticket reduce) pick exactly the token of the
    one-workgroup kernel (same per-index noise); top-k / top-p rows keep the whole-row path. Three launches check
    that the tickets re-arm."""
    from kafka_llm_service_amd.ops._ext import ext

    torch.manual_seed(14)
    B, V = 64, 128256
    logits = torch.randn(B, V, device=cuda).to(torch.bfloat16)
    temp = torch.tensor([0.0, 0.7, 1.3, 0.7] * (B // 4), device=cuda)
    topp = torch.tensor([1.0, 1.0, 1.0, 0.9] * (B // 4), device=cuda)
    topk = torch.tensor([0, 0, 0, 50] * (B // 4), dtype=torch.int32, device=cuda)
    seeds = torch.arange(B, dtype=torch.long, device=cuda) * 7 + 3
    step = torch.tensor([5], dtype=torch.long, device=cuda)
    one = torch.empty(B, dtype=torch.long, device=cuda)
    ext().sample(logits, temp, topp, topk, seeds, step, one, None, 1)
    for it in range(3):
        split = ops.sample(logits, temp, topp, topk, seeds, step)
        assert torch.equal(split.cpu(), one.cpu()), f"launch {it}"
    assert torch.equal(one[0::4].cpu(), logits[0::4].float().argmax(-1).cpu())


def test_attn_merge_ignores_unwritten_slots(cuda):
    """Rows with fewer pieces than the partial buffer's S: their extra slots keep lse = -inf and whatever bytes the
    allocator left there (NaN here) — the merge must not turn 0 x NaN into NaN."""
    torch.manual_seed(15)
    rows, Hq, S, D = 40, 32, 4, 128
    part = torch.randn(rows, Hq, S, D, device=cuda)
    lse = torch.randn(rows, Hq, S, device=cuda)
    part[::2, :, 2:] = float("nan")
    lse[::2, :, 2:] = float("-inf")
    out = torch.empty(rows, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.attn_merge(part, lse, out)
    ref_out = torch.empty(rows, Hq, D, dtype=torch.bfloat16)
    ref.attn_merge(part.cpu(), lse.cpu(), ref_out)
    assert torch.isfinite(out.float()).all() and torch.isfinite(ref_out.float()).all()
    _close(out, ref_out, atol=0.02, msg="merge with unwritten slots")


@pytest.mark.parametrize("T,ep,E,k", [(37, 2, 8, 2), (64, 4, 8, 2), (5, 8, 8, 2)])
def test_ep_dispatch_route_combine_match_reference(cuda, T, ep, E, k):
    """csrc/moe.hip ep_dispatch / ep_recv_route / ep_combine == the fp32/host references of the same image layout
    (rows, metadata, slot maps, expert-sorted routing bit-exact; combine to bf16 rounding), with the all-to-all
    simulated by re-stacking the ranks' images."""
    from kafka_llm_service_amd import ops

    torch.manual_seed(T + ep)
    d = 256
    El = E // ep
    x = torch.randn(T, d, device="cuda", dtype=torch.bfloat16)
    r = ops.moe_route(torch.randn(T, E, device="cuda", dtype=torch.bfloat16), k)
    Tl, C, MR = ops.ep_layout(T, ep, k, El, d)
    imgs, slots = [], []
    for q in range(ep):
        lo, hi = min(T, q * Tl), min(T, (q + 1) * Tl)
        img, slot = ops.ep_dispatch(x, r.topk_e, lo, hi - lo, El, ep, C, MR)
        rimg, rslot = ops.ep_dispatch(x.cpu(), r.topk_e.cpu(), lo, hi - lo, El, ep, C, MR)
        for p in range(ep):
            meta, rmeta = img[p, C:].reshape(-1).view(torch.int32).cpu(), rimg[p, C:].reshape(-1).view(torch.int32)
            n = int(rmeta[0])
            assert int(meta[0]) == n and torch.equal(meta[4:4 + C], rmeta[4:4 + C])
            assert torch.equal(img[p, :n].cpu(), rimg[p, :n])
        assert torch.equal(slot[:(hi - lo) * k].cpu(), rslot[:(hi - lo) * k])
        imgs.append(img)
        slots.append(slot)
    for p in range(ep):  # rank p's received image: block s = rank s's part for p
        recv = torch.stack([imgs[s][p] for s in range(ep)])
        rr = ops.ep_recv_route(recv, C, El)
        ref = ops.ep_recv_route(recv.cpu(), C, El)
        n = int(ref.expert_off[-1])
        assert torch.equal(rr.expert_off.cpu(), ref.expert_off) and torch.equal(rr.tile_off.cpu(), ref.tile_off)
        assert torch.equal(rr.perm_tok[:n].cpu(), ref.perm_tok[:n])
        assert torch.all(rr.perm_w[:n].cpu() == 1) and torch.all(rr.perm_tok[n:].cpu() == 0)
    for q in range(ep):  # combine over a synthetic returned image
        lo, hi = min(T, q * Tl), min(T, (q + 1) * Tl)
        back = torch.randn(ep, C + MR, d, device="cuda", dtype=torch.bfloat16)
        out = torch.zeros(Tl, d, device="cuda", dtype=torch.bfloat16)
        ops.ep_combine(back, slots[q], r.topk_w, lo, hi - lo, out)
        ref_out = torch.zeros(Tl, d, dtype=torch.bfloat16)
        ops.ep_combine(back.cpu(), slots[q].cpu(), r.topk_w.cpu(), lo, hi - lo, ref_out)
        torch.testing.assert_close(out.cpu().float(), ref_out.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [130, 168, 200, 256])
@pytest.mark.parametrize("shape", [("qkv", 6144, 4096, False), ("o", 4096, 4096, False),
                                   ("gate_up", 2 * 14336, 4096, True), ("down", 4096, 14336, False)],
                         ids=lambda s: s[0] if isinstance(s, tuple) else str(s))
def test_skinny_gemm_matches_fp32(cuda, M, shape):
    """csrc/skinny_gemm.hip (129..256 rows, LDS-DMA ring, 2x2 MFMA tiles per wave) == fp32 X . W^T on the
    Llama-3-8B projection shapes, split-K slabs summed; gate_up with the fused SwiGLU epilogue."""
    from kafka_llm_service_amd import ops
    from kafka_llm_service_amd.ops import reference as ref

    _, N, K, glu = shape
    torch.manual_seed(M + N)
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wt = ops.tile_weight(w, glu=glu)
    y = ops.linear_skinny(x, wt, glu=glu)
    want = x.float() @ w.float().t()
    if glu:
        want = ref.silu_mul(want)
        if ops.is_slab(y):
            y = ref.silu_mul(y.sum(0))
    elif ops.is_slab(y):
        y = y.sum(0)
    torch.testing.assert_close(y.float(), want, atol=2e-2, rtol=2e-2)


def test_sample_proc_matches_reference(cuda):
    """The sampler's device-side logits processing (csrc/sampling.hip RowProc, engine/logits_proc.py) against
    ops.reference: grammar bitmask rows (greedy = the masked argmax; temperature / top-p draws stay inside the mask),
    forced rows, presence / frequency penalties read from and written to the count table, split rows included."""
    from kafka_llm_service_amd.engine.logits_proc import LogitsProcessor
    from kafka_llm_service_amd.engine.sequence import SamplingParams, Sequence

    torch.manual_seed(21)
    B, V = 24, 128256
    logits = (torch.randn(B, V, device=cuda) * 3).to(torch.bfloat16)
    lp_g = LogitsProcessor(cuda, V, max_slots=32, mask_rows=16)
    lp_c = LogitsProcessor("cpu", V, max_slots=32, mask_rows=16)
    seqs = [Sequence(f"r{i}", [1], SamplingParams(temperature=0.0, presence_penalty=0.4 * (i % 3 == 2),
                                                  frequency_penalty=1.5 * (i % 3 == 2))) for i in range(B)]
    g = torch.Generator().manual_seed(3)
    rows = []
    for i in range(B):
        if i % 4 == 0:
            rows.append((i, seqs[i], torch.randint(0, V, (int(torch.randint(2, 3000, (1,), generator=g)),),
                                                   generator=g).tolist()))
        elif i % 4 == 1:
            rows.append((i, seqs[i], [int(torch.randint(0, V, (1,), generator=g))]))
        elif i % 3 == 2:
            rows.append((i, seqs[i], None))
    proc, upd = lp_g.build(rows, B)
    proc_c, upd_c = lp_c.build(rows, B)
    assert (proc == proc_c).all()
    lp_g.apply(upd, lambda a: torch.from_numpy(a).to(cuda))
    lp_c.apply(upd_c, torch.from_numpy)
    mt_g, cnt_g = lp_g.tables()
    mt_c, cnt_c = lp_c.tables()
    assert torch.equal(mt_g.cpu(), mt_c)
    pd = torch.from_numpy(proc).to(cuda)
    for step in range(4):  # greedy: bitwise the reference's pick (counts evolve identically)
        tok = ops.sample(logits, torch.zeros(B, device=cuda), proc=pd, mask_tab=mt_g, counts=cnt_g)
        ref_tok = ref.sample(logits.cpu(), torch.zeros(B), proc=torch.from_numpy(proc), mask_tab=mt_c,
                             counts=cnt_c)
        assert torch.equal(tok.cpu(), ref_tok), f"step {step}"
        assert torch.equal(cnt_g.cpu(), cnt_c), f"counts after step {step}"
    # temperature (split rows) and top-p (whole-row sampler): every draw obeys the row's mask / forced id
    seeds = torch.arange(B, dtype=torch.long, device=cuda) * 13 + 1
    x, forced = ref.process_logits(logits.cpu(), torch.from_numpy(proc), mt_c, cnt_c)
    allowed = torch.isfinite(x)
    for topp in (1.0, 0.9):
        for s in range(3):
            tok = ops.sample(logits, torch.full((B,), 0.9, device=cuda), torch.full((B,), topp, device=cuda),
                             None, seeds + s, proc=pd, mask_tab=mt_g, counts=cnt_g).cpu()
            for i in range(B):
                if forced[i] >= 0:
                    assert int(tok[i]) == int(forced[i])
                else:
                    assert bool(allowed[i, int(tok[i])]), (i, int(tok[i]))


def test_cascade_pass_with_new_turn_rows(cuda):
    """The cascade prefix pass over decode rows AND a new turn's prefill rows in ONE launch (tile v3, items flagged
    alt write fp32 partials into the prefill merge buffer at row token - B), then the new turn's own tiles over the
    keys behind the prefix (slots from nc on) and the merge: the new turn's rows equal fp32 causal attention over
    their whole context, and the decode rows' bf16 prefix partials are bitwise those of a pass without the new
    turn."""
    torch.manual_seed(14)
    Hq, Hkv, D = 32, 8, 128
    G = Hq // Hkv
    P, hist, Tn = 1024, 200, 70  # shared prefix, the new turn's own history, new-turn tokens
    B = 5
    g = torch.Generator().manual_seed(15)
    n_pref = P // 16
    ctx = P + hist + Tn
    nb_total = n_pref + B * 4 + (ctx - P) // 16 + 4
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16).to(cuda)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16).to(cuda)
    bt = torch.zeros(B + 1, 128, dtype=torch.int32)
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        bt[b, n_pref:n_pref + 4] = torch.arange(n_pref + 4 * b, n_pref + 4 * b + 4)
    nn = -(-(ctx - P) // 16)
    bt[B, :n_pref] = torch.arange(n_pref)
    bt[B, n_pref:n_pref + nn] = torch.arange(n_pref + 4 * B, n_pref + 4 * B + nn)
    bt = bt.to(cuda)
    T = B + Tn
    q = torch.randn(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    a = P + hist  # first new-turn position
    q_limit = torch.cat([torch.full((B,), P + 40, dtype=torch.int32), torch.arange(a, a + Tn, dtype=torch.int32)])
    q_limit = q_limit.to(cuda)
    scale = 1 / math.sqrt(D)
    nc, ck = 4, P // 4
    tile = 256 // G
    pre_items = [(0, B, 0, c * ck, (c + 1) * ck, c, 0, 0) for c in range(nc)]
    alt_items = [(B + t0, min(tile, Tn - t0), 0, c * ck, (c + 1) * ck, c, 1, 0)
                 for c in range(nc) for t0 in range(0, Tn, tile)]
    S_dec, S_new = nc + 1, nc + 3
    pre_a = torch.zeros(B, Hq, S_dec, D, device=cuda, dtype=torch.bfloat16)
    lse_a = torch.zeros(B, Hq, S_dec, device=cuda)
    pre_b, lse_b = pre_a.clone(), lse_a.clone()
    part_new = torch.zeros(Tn, Hq, S_new, D, device=cuda)
    lse_new = torch.full((Tn, Hq, S_new), float("-inf"), device=cuda)
    it_all = torch.tensor(pre_items + alt_items, dtype=torch.int32, device=cuda)
    ops.attn_prefill(it_all, q, k, v, bt, q_limit, scale, out_part=pre_a, lse_part=lse_a, variant=3,
                     alt_part=part_new, alt_lse=lse_new, alt_tok_off=B)
    ops.attn_prefill(torch.tensor(pre_items, dtype=torch.int32, device=cuda), q[:B], k, v, bt, q_limit, scale,
                     out_part=pre_b, lse_part=lse_b, variant=3)
    torch.cuda.synchronize()
    assert torch.equal(pre_a, pre_b) and torch.equal(lse_a, lse_b)
    # the new turn's own keys [P, ctx) in 3 pieces, slots nc.., rows relative to B
    own = [(t0, min(tile, Tn - t0), B, P + c * 160, min(ctx, P + (c + 1) * 160), nc + c, 0, 0)
           for t0 in range(0, Tn, tile) for c in range(3)]
    ops.attn_prefill(torch.tensor(own, dtype=torch.int32, device=cuda), q[B:], k, v, bt, q_limit[B:], scale,
                     out_part=part_new, lse_part=lse_new, variant=3)
    out = torch.empty(Tn, Hq, D, device=cuda, dtype=torch.bfloat16)
    ops.attn_merge(part_new, lse_new, out)
    # fp32 reference: causal attention of each new-turn token over its whole context through block-table row B
    kk, vv = ref.gather_kv(k.cpu(), v.cpu(), bt[B].cpu(), ctx)
    o_ref = torch.empty(Tn, Hq, D)
    for t in range(Tn):
        pos = a + t
        for h in range(Hkv):
            qs = q[B + t, h * G:(h + 1) * G].float().cpu()
            s_ = (qs @ kk[:pos + 1, h].float().t()) * scale
            p_ = torch.softmax(s_, -1)
            o_ref[t, h * G:(h + 1) * G] = p_ @ vv[:pos + 1, h].float()
    _close(out, o_ref, atol=0.02, msg="new-turn rows through the cascade pass")
