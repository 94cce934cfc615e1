"""Buffers written with sc1 (write-through, agent-scope) stores, each rewritten round after round after readers on
every XCD cached its previous contents — the engine's layer-after-layer pattern — and checked against fp32 every round
(common.h "Store / load scopes"). One test per kept sc1 site not covered by test_kernels_gpu.py's slab tests:
GEMM bf16 outputs (fused SwiGLU, lm_head), cascade bf16 prefix partials, decode ticket-merge partial rows."""
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


@pytest.mark.parametrize("M", [17, 64, 128])
def test_wstream_glu_output_reused_buffer(cuda, M):
    """gate_up with its fused SwiGLU (one split, bf16 Y through the workgroup LDS tile as 16-B sc1 stores): ONE Y
    buffer rewritten six times; between rounds a torch reduction and the down projection (our GEMM, every XCD) read
    it."""
    ext = ops._ext.load()
    N, K, F = 28672, 4096, 14336
    g = torch.Generator(device=cuda).manual_seed(3)
    w = (torch.randn(N, K, device=cuda, generator=g) * K ** -0.5).to(torch.bfloat16)
    wt = ops.tile_weight(w, glu=True)
    wd = (torch.randn(K, F, device=cuda, generator=g) * F ** -0.5).to(torch.bfloat16)
    wdt = ops.tile_weight(wd)
    assert ops.stream_plan(M, N, K)[2] == 1
    y = torch.empty(M, F, device=cuda, dtype=torch.bfloat16)
    for it in range(6):
        x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, generator=g)
        ext.wstream_gemm(x, wt, y, None, 8, True, True)
        y_ref = ref.silu_mul(x.float() @ w.float().t())
        _close(y, y_ref, atol=0.03, rtol=0.02, msg=f"glu round {it}")
        _ = y.float().sum().item()                       # torch readers
        d = ops.slab_reduce(ops.linear_stream(y, wdt))   # our GEMM reading y on every XCD
        _close(d, y.float() @ wd.float().t(), atol=0.03, rtol=0.02, msg=f"down of y round {it}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("M", [1, 64])
def test_lm_head_output_reused_buffer(cuda, M):
    """lm_head (un-split bf16 logits, 16-B sc1 stores): ONE logits buffer rewritten six times, read by torch and by the
    sampler kernel between rounds; greedy ids must be the fp32 argmax wherever it is unambiguous."""
    ext = ops._ext.load()
    V, K = 128256, 4096
    g = torch.Generator(device=cuda).manual_seed(4)
    w = (torch.randn(V, K, device=cuda, generator=g) * K ** -0.5).to(torch.bfloat16)
    wt = ops.tile_weight(w)
    logits = torch.empty(M, V, device=cuda, dtype=torch.bfloat16)
    for it in range(6):
        x = torch.randn(M, K, device=cuda, dtype=torch.bfloat16, generator=g)
        ext.wstream_gemm(x, wt, logits, None, 1, True, False)
        ref_l = torch.cat([x.float() @ w[i:i + 16384].float().t() for i in range(0, V, 16384)], 1)
        _close(logits, ref_l, atol=0.03, rtol=0.01, msg=f"lm_head round {it}")
        ids = ops.sample(logits)                          # sampler kernel reads the buffer
        top2 = ref_l.topk(2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 0.05
        assert torch.equal(ids[clear].cpu(), ref_l.argmax(1)[clear].cpu()), f"greedy ids round {it}"
        _ = logits.float().sum().item()
    torch.cuda.synchronize()


def _paged_prefix_case(cuda, Hkv, P, suffix, seed):
    D = 128
    B = len(suffix)
    lens = [P + s for s in suffix]
    n_pref = P // 16
    nb_total = n_pref + sum((s + 15) // 16 + 1 for s in suffix) + 2
    g = torch.Generator().manual_seed(seed)
    k = torch.randn(nb_total, Hkv, 16, D, generator=g).to(torch.bfloat16).to(cuda)
    v = torch.randn(nb_total, Hkv, D, 16, generator=g).to(torch.bfloat16).to(cuda)
    W = max((L + 15) // 16 for L in lens)
    bt = torch.zeros(B, W, dtype=torch.int32)
    c = n_pref
    for b in range(B):
        bt[b, :n_pref] = torch.arange(n_pref)
        n = (lens[b] + 15) // 16 - n_pref
        bt[b, n_pref:n_pref + n] = torch.arange(c, c + n)
        c += n
    return k, v, bt.to(cuda), lens


def test_cascade_bf16_partials_reused_buffer(cuda):
    """Cascade prefix pass (tile v3) writing bf16 partials as 16-B sc1 stores into ONE partial buffer, then the
    suffix decode with the fused merge reading them; six rounds with new queries, torch reading the partials between
    rounds. Every round == dense attention."""
    torch.manual_seed(7)
    Hq, Hkv, D, P = 32, 8, 128, 16 * 24
    suffix = [1, 40, 300, 77, 5, 129]
    B = len(suffix)
    k, v, bt, lens = _paged_prefix_case(cuda, Hkv, P, suffix, 8)
    n_pre, S = 4, 2
    part = torch.empty(B, Hq, n_pre + S, D, device=cuda)
    pre = torch.empty(B, Hq, n_pre + S, D, device=cuda, dtype=torch.bfloat16)
    lse = torch.empty(B, Hq, n_pre + S, device=cuda)
    bounds = [round(P * i / n_pre / 32) * 32 for i in range(n_pre)] + [P]
    items = torch.tensor([[0, B, 0, bounds[i], bounds[i + 1], i, 0, 0] for i in range(n_pre)], dtype=torch.int32,
                         device=cuda)
    q_limit = torch.full((B,), 1 << 30, dtype=torch.int32, device=cuda)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    ks = torch.full((B,), P, dtype=torch.int32, device=cuda)
    dit = ops.uniform_decode_items(sl, ks, S, n_pre)
    scale = 1 / math.sqrt(D)
    for it in range(6):
        q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
        ops.attn_prefill(items, q, k, v, bt, q_limit, scale, out_part=pre, lse_part=lse, variant=3)
        out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode_items(q, k, v, bt, dit, part, lse, scale, out=out, pre_part=pre)
        o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
        _close(out, o_ref, atol=0.03, msg=f"cascade bf16 partials round {it}")
        _ = (pre.float().sum() + part.sum()).item()  # readers on every XCD cache the partial lines
    torch.cuda.synchronize()


@pytest.mark.parametrize("S", [4, 16])
def test_ticket_merge_partials_reused_buffer(cuda, S):
    """Split suffix decode: each split's partial row leaves as 16-B sc1 stores and the last split reads them back with
    sc1 loads (compiler-tracked buffer loads) in the same launch. ONE partial buffer, six rounds, torch reading it
    between rounds; every round == dense attention."""
    torch.manual_seed(9)
    Hq, Hkv, D = 32, 8, 128
    suffix = [700, 1900, 33, 64, 2500]
    B = len(suffix)
    k, v, bt, lens = _paged_prefix_case(cuda, Hkv, 0, suffix, 10)
    sl = torch.tensor(lens, dtype=torch.int32, device=cuda)
    part = torch.empty(B, Hq, S, D, device=cuda)
    lse = torch.empty(B, Hq, S, device=cuda)
    scale = 1 / math.sqrt(D)
    for it in range(6):
        q = torch.randn(B, Hq, D, device=cuda, dtype=torch.bfloat16)
        out = torch.full((B, Hq, D), float("nan"), device=cuda, dtype=torch.bfloat16)
        ops.attn_decode(q, k, v, bt, sl, None, part, lse, S, 0, scale, out=out)
        o_ref, _ = ref.attn_decode_full(q.cpu(), k.cpu(), v.cpu(), bt.cpu(), sl.cpu(), scale)
        _close(out, o_ref, atol=0.02, msg=f"ticket merge S={S} round {it}")
        _ = (part.sum() + lse.sum()).item()
    torch.cuda.synchronize()


@pytest.mark.parametrize("T", [1, 64])
def test_norm_rope_attn_outputs_reused_buffers(cuda, T):
    """The layer chain's small kernels with their default 16-B sc1 stores, on ONE set of buffers rewritten six times
    (the engine's layer after layer): fused_add_rmsnorm (normalised rows + the in-place residual), rope_kv_write (q rows
    and the K cache rows) and the decode kernel's final bf16 rows (through LDS, decode_piece OST). Between rounds torch
    and our decode GEMM (every XCD) read each buffer; every round is checked against fp32 references."""
    g = torch.Generator(device=cuda).manual_seed(11)
    d, Hq, Hkv, D = 4096, 32, 8, 128
    nb = 20 * T  # 20 pages per row, none shared
    eps = 1e-5
    wn = (1 + 0.1 * torch.randn(d, device=cuda, generator=g)).to(torch.bfloat16)
    wo = (torch.randn(d, d, device=cuda, generator=g) * d ** -0.5).to(torch.bfloat16)
    wot = ops.tile_weight(wo)
    cs = ref.rope_cos_sin(8192, D, 500000.0, None, device=cuda)
    resid = torch.randn(T, d, device=cuda, dtype=torch.bfloat16, generator=g)
    x = torch.empty(T, d, device=cuda, dtype=torch.bfloat16)
    q = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    kc = torch.zeros(nb, Hkv, 16, D, device=cuda, dtype=torch.bfloat16)
    vc = torch.zeros(nb, Hkv, D, 16, device=cuda, dtype=torch.bfloat16)
    out = torch.empty(T, Hq, D, device=cuda, dtype=torch.bfloat16)
    L = 16 * 20  # keys per row: 20 pages of its own
    bt = torch.arange(T * 20, dtype=torch.int32, device=cuda).view(T, 20)
    lens = torch.full((T,), L, dtype=torch.int32, device=cuda)
    S = 2
    part = torch.empty(T, Hq, S, D, device=cuda)
    lse = torch.empty(T, Hq, S, device=cuda)
    dit = ops.uniform_decode_items(lens, None, S, 0)
    for it in range(6):
        delta = torch.randn(T, d, device=cuda, dtype=torch.bfloat16, generator=g)
        r0 = resid.clone()
        ops.fused_add_rmsnorm(delta, resid, wn, eps, out=x)
        y_ref, s_ref = ref.fused_add_rmsnorm(delta.cpu(), r0.cpu(), wn.cpu(), eps)
        _close(resid, s_ref, atol=0.0, msg=f"residual round {it}")
        _close(x, y_ref, atol=0.02, rtol=0.01, msg=f"rmsnorm round {it}")
        # readers: torch and the decode GEMM on every XCD
        _ = (x.float().sum() + resid.float().sum()).item()
        _close(ops.slab_reduce(ops.linear_stream(x, wot)), x.float() @ wo.float().t(), atol=0.03, rtol=0.02,
               msg=f"gemm of x round {it}")
        # RoPE + KV write: every row writes its key at a new position of its own pages
        qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=cuda, dtype=torch.bfloat16, generator=g)
        pos = torch.full((T,), it, dtype=torch.long, device=cuda)
        slots = (bt[:, it // 16].long() * 16 + it % 16)
        kc_ref, vc_ref = kc.cpu().clone(), vc.cpu().clone()
        ops.rope_kv_write(qkv, pos, cs, q, kc, vc, slots, Hq, Hkv)
        q_ref = torch.empty(T, Hq, D, dtype=torch.bfloat16)
        ref.rope_kv_write(qkv.cpu(), pos.cpu(), cs.cpu(), q_ref, kc_ref, vc_ref, slots.cpu(), Hq, Hkv)
        _close(q, q_ref, atol=0.03, rtol=0.01, msg=f"q round {it}")
        _close(kc, kc_ref, atol=0.03, rtol=0.01, msg=f"k cache round {it}")
        assert torch.equal(vc.cpu(), vc_ref), f"v cache round {it}"
        _ = (q.float().sum() + kc.float().sum()).item()
        # decode over the rows' pages (keys written so far and zeros beyond: both are keys), one output buffer
        ops.attn_decode_items(q, kc, vc, bt, dit, part, lse, D ** -0.5, out=out)
        o_ref, _ = ref.attn_decode_full(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens.cpu(), D ** -0.5)
        _close(out, o_ref, atol=0.03, msg=f"decode out round {it}")
        _close(ops.slab_reduce(ops.linear_stream(out.view(T, -1), wot)), out.view(T, -1).float() @ wo.float().t(),
               atol=0.03, rtol=0.02, msg=f"gemm of decode out round {it}")
    torch.cuda.synchronize()
