"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

They define the numerics the CDNA4 kernels are tested against, and they are the CPU execution path used by the
unit tests (no GPU in CI). They use exactly the same tensor layouts as the kernels, including the paged KV layout
  K page: [num_blocks, Hkv, 16, D] holding D/8 chunk planes [D/8][16 keys][8] (k_planes / k_natural below)
  V page: [num_blocks, Hkv, D, 16]  (V^T, key offset o at vt_pos(o)).
or, for the fp8 cache (kv_dtype="fp8", ops/csrc/rope_kv.hip), uint8 pages
  K page: [num_blocks, Hkv, 16 * D + 32]: e4m3 units [D/32 j][2 h][16 keys][2 s][8 e] holding d = 32j + 16s + 8h + e,
          then int8 exponents: K of key o at 16D + o, V of key o at 16D + 16 + vt_pos(o) (value = e4m3 * 2^e)
  V page: [num_blocks, Hkv, D * 16]: e4m3 V^T [D][16], key o at vt_pos(o).
"""
from __future__ import annotations

import math

import torch

PAGE = 16
LOG2E = 1.4426950408889634


def vt_pos(o: torch.Tensor | int):
    """Position of key offset ``o`` inside a V^T page (swap bits 2 and 3)."""
    if isinstance(o, int):
        return (o & ~15) | (o & 3) | ((o & 4) << 1) | ((o & 8) >> 1)
    return (o & ~15) | (o & 3) | ((o & 4) << 1) | ((o & 8) >> 1)


_VT_PERM = torch.tensor([vt_pos(o) for o in range(PAGE)], dtype=torch.long)


FP8_MAX = 448.0
FP8_EXP_MIN, FP8_EXP_MAX = -100, 100


def is_fp8_cache(k_cache: torch.Tensor) -> bool:
    return k_cache.dtype == torch.uint8


def cache_head_dim(k_cache: torch.Tensor, v_cache: torch.Tensor) -> int:
    return v_cache.shape[-1] // PAGE if is_fp8_cache(k_cache) else k_cache.shape[-1]


def kv_cache_shapes(num_blocks: int, hkv: int, D: int, kv_dtype: str = "bf16"):
    """(K shape, V shape, torch dtype) of one layer's paged cache."""
    if kv_dtype == "fp8":
        return (num_blocks, hkv, PAGE * D + 32), (num_blocks, hkv, D * PAGE), torch.uint8
    if kv_dtype != "bf16":
        raise ValueError(f"kv_dtype must be bf16 or fp8, not {kv_dtype!r}")
    return (num_blocks, hkv, PAGE, D), (num_blocks, hkv, D, PAGE), torch.bfloat16


def kv_page_bytes(hkv: int, D: int, kv_dtype: str = "bf16") -> int:
    """Bytes of K + V for one 16-token page of one layer."""
    return hkv * (2 * PAGE * D + 32) if kv_dtype == "fp8" else hkv * 2 * PAGE * D * 2


def fp8_quant(x: torch.Tensor):
    """Per-vector e4m3 quantization over the last dim: (bytes uint8 [..., D], exponent int [...]) with
    x ~= e4m3(bytes) * 2^e and e = frexp exponent of amax / 448 (the kernel's rule, rope_kv.hip)."""
    x = x.float()
    amax = x.abs().amax(-1)
    _, e = torch.frexp(amax / FP8_MAX)
    e = torch.where(amax > 0, e, torch.zeros_like(e)).clamp(FP8_EXP_MIN, FP8_EXP_MAX)
    y = torch.ldexp(x, -e[..., None].float()).clamp(-FP8_MAX, FP8_MAX)
    return y.to(torch.float8_e4m3fn).view(torch.uint8), e


def fp8_dequant_pages(k_pages: torch.Tensor, v_pages: torch.Tensor):
    """fp8 pages (K [n, Hkv, 16D + 32], V [n, Hkv, 16D] uint8) -> fp32 K [n, Hkv, 16, D] and V [n, Hkv, D, 16]
    (V in natural key order)."""
    n, hkv = k_pages.shape[:2]
    D = v_pages.shape[-1] // PAGE
    data = k_pages[..., :PAGE * D].contiguous().view(torch.float8_e4m3fn).float()
    k = data.view(n, hkv, D // 32, 2, PAGE, 2, 8).permute(0, 1, 4, 2, 5, 3, 6).reshape(n, hkv, PAGE, D)
    ke = k_pages[..., PAGE * D:PAGE * D + PAGE].contiguous().view(torch.int8).float()
    ve = k_pages[..., PAGE * D + PAGE:PAGE * D + 2 * PAGE].contiguous().view(torch.int8).float()
    k = k * torch.exp2(ke)[..., None]
    v = v_pages.contiguous().view(torch.float8_e4m3fn).float().view(n, hkv, D, PAGE) * torch.exp2(ve)[:, :, None, :]
    return k, v[..., _VT_PERM.to(v.device)]


def fp8_pack_pages(k: torch.Tensor, v: torch.Tensor):
    """Natural-order K, V [n, Hkv, 16, D] -> fp8 pages (K [n, Hkv, 16D + 32], V [n, Hkv, 16D] uint8), every
    (key, head) vector quantized on its own (the layout rope_kv_write produces)."""
    n, hkv, _, D = k.shape
    kq, ke = fp8_quant(k)
    vq, ve = fp8_quant(v)
    kp = torch.zeros(n, hkv, PAGE * D + 2 * PAGE, dtype=torch.uint8, device=k.device)
    kp[..., :PAGE * D] = kq.view(n, hkv, PAGE, D // 32, 2, 2, 8).permute(0, 1, 3, 5, 2, 4, 6).reshape(n, hkv, -1)
    kp[..., PAGE * D:PAGE * D + PAGE] = ke.to(torch.int8).view(torch.uint8)
    perm = _VT_PERM.to(k.device)
    kp[..., PAGE * D + PAGE + perm] = ve.to(torch.int8).view(torch.uint8)
    vt = torch.zeros(n, hkv, D, PAGE, dtype=torch.uint8, device=k.device)
    vt[..., perm] = vq.transpose(2, 3)
    return kp, vt.reshape(n, hkv, D * PAGE)


def k_planes(k_cache: torch.Tensor) -> torch.Tensor:
    """View of a K cache [nb, Hkv, 16, D] as its chunk planes [nb, Hkv, D/8, 16 keys, 8] (the memory layout)."""
    nb, hkv, _, D = k_cache.shape
    return k_cache.view(nb, hkv, D // 8, PAGE, 8)


def k_natural(k_pages: torch.Tensor) -> torch.Tensor:
    """K pages [n, Hkv, 16, D] as stored -> [n, Hkv, 16 keys, D] in natural (key, d) order."""
    n, hkv, _, D = k_pages.shape
    return k_pages.reshape(n, hkv, D // 8, PAGE, 8).permute(0, 1, 3, 2, 4).reshape(n, hkv, PAGE, D)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    s = (x.float() + residual.float()).to(residual.dtype)
    return rmsnorm(s, w, eps), s


def silu_mul(x: torch.Tensor) -> torch.Tensor:
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def rope_kv_write(qkv, positions, cos_sin, q_out, k_cache, v_cache, slot_mapping, Hq: int, Hkv: int) -> None:
    T = qkv.shape[0]
    D = cache_head_dim(k_cache, v_cache)
    half = D // 2
    x = qkv.float().view(T, Hq + 2 * Hkv, D)
    cs = cos_sin[positions.long()].float()  # [T, D]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    qk = x[:, : Hq + Hkv]
    x1, x2 = qk[..., :half], qk[..., half:]
    rot32 = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)
    rot = rot32.to(qkv.dtype)
    q_out.copy_(rot[:, :Hq])
    if slot_mapping is None:
        return
    if is_fp8_cache(k_cache):
        kq, ke = fp8_quant(rot32[:, Hq:])
        vq, ve = fp8_quant(x[:, Hq + Hkv:])
        kd = kq.view(T, Hkv, D // 32, 2, 2, 8).permute(0, 1, 2, 4, 3, 5)  # (j, s, h, e) -> (j, h, s, e)
        for t in range(T):
            s = int(slot_mapping[t])
            if s < 0:
                continue
            blk, off = divmod(s, PAGE)
            k_cache[blk, :, :PAGE * D].view(Hkv, D // 32, 2, PAGE, 2, 8)[:, :, :, off] = kd[t]
            k_cache[blk, :, PAGE * D + off] = ke[t].to(torch.int8).view(torch.uint8)
            k_cache[blk, :, PAGE * D + PAGE + vt_pos(off)] = ve[t].to(torch.int8).view(torch.uint8)
            v_cache[blk].view(Hkv, D, PAGE)[:, :, vt_pos(off)] = vq[t]
        return
    k = rot[:, Hq:]
    v = x[:, Hq + Hkv:].to(qkv.dtype)
    for t in range(T):
        s = int(slot_mapping[t])
        if s < 0:
            continue
        blk, off = divmod(s, PAGE)
        k_planes(k_cache)[blk, :, :, off, :] = k[t].reshape(Hkv, D // 8, 8)
        v_cache[blk, :, :, vt_pos(off)] = v[t]


def gather_kv(k_cache, v_cache, block_table, length: int):
    """Materialise [length, Hkv, D] K and V for one sequence from the paged caches (fp32)."""
    nb = (length + PAGE - 1) // PAGE
    ids = block_table[:nb].long()
    if is_fp8_cache(k_cache):
        k, v = fp8_dequant_pages(k_cache[ids], v_cache[ids])
    else:
        k = k_natural(k_cache[ids].float())  # [nb, Hkv, 16, D]
        v = v_cache[ids].float()  # [nb, Hkv, D, 16]
        v = v[..., _VT_PERM.to(v.device)]  # undo the page permutation -> [nb, Hkv, D, 16] natural key order
    k = k.permute(0, 2, 1, 3).reshape(nb * PAGE, k.shape[1], k.shape[3])[:length]
    v = v.permute(0, 3, 1, 2).reshape(nb * PAGE, v.shape[1], v.shape[2])[:length]
    return k, v


def _attend(q, k, v, mask, scale):
    """q [M, G, D], k/v [N, D] (one kv head), mask [M, N] bool -> (o [M, G, D], lse2 [M, G])."""
    s = torch.einsum("mgd,nd->mgn", q, k) * scale
    s = s.masked_fill(~mask[:, None, :], float("-inf"))
    m = s.amax(-1, keepdim=True)
    m_use = torch.where(torch.isinf(m), torch.zeros_like(m), m)
    p = torch.exp(s - m_use)
    l = p.sum(-1, keepdim=True)
    o = torch.einsum("mgn,nd->mgd", p, v) / torch.where(l > 0, l, torch.ones_like(l))
    lse = torch.where(l[..., 0] > 0, (m_use[..., 0] + torch.log(l[..., 0])) * LOG2E,
                      torch.full_like(l[..., 0], float("-inf")))
    return o, lse


def attn_decode_full(q, k_cache, v_cache, block_tables, seq_lens, scale, kv_start=None):
    """Reference single-token paged attention over keys [kv_start, seq_len). q [B, Hq, D] -> (o fp32, lse2)."""
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    out = torch.zeros(B, Hq, D, dtype=torch.float32, device=q.device)
    lse = torch.full((B, Hq), float("-inf"), dtype=torch.float32, device=q.device)
    for b in range(B):
        L = int(seq_lens[b])
        s0 = int(kv_start[b]) if kv_start is not None else 0
        if L <= s0:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[b], L)
        for h in range(Hkv):
            qh = q[b, h * G:(h + 1) * G].float()[None]
            mask = torch.zeros(1, L, dtype=torch.bool, device=q.device)
            mask[:, s0:L] = True
            o, l2 = _attend(qh, k[:, h], v[:, h], mask, scale)
            out[b, h * G:(h + 1) * G] = o[0]
            lse[b, h * G:(h + 1) * G] = l2[0]
    return out, lse


def attn_decode_items(q, k_cache, v_cache, block_tables, items, out_part, lse_part, scale, out=None,
                      pre_part=None):
    """Reference for the work-item decode kernel (ops/csrc/attention.hip attn_decode_kernel). ``pre_part`` (bf16,
    out_part's shape): the cascade's prefix partials (slots < npre) are read from it instead of out_part."""
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    S_total = out_part.shape[2]
    lp = lse_part.view(out_part.shape[0], Hq, S_total)
    nparts, npres = {}, {}
    for b, lo, hi, split, nsplit, npre in (it[:6] for it in items.tolist()):
        if not (0 <= b < B and 0 <= split < nsplit and npre >= 0 and npre + nsplit <= S_total):
            continue  # padding / malformed item: dropped, as by the kernel
        nparts[b] = npre + nsplit
        npres[b] = npre
        o = torch.zeros(Hq, D, dtype=torch.float32, device=q.device)
        l2 = torch.full((Hq,), float("-inf"), dtype=torch.float32, device=q.device)
        if hi > lo:
            k, v = gather_kv(k_cache, v_cache, block_tables[b], hi)
            mask = torch.zeros(1, hi, dtype=torch.bool, device=q.device)
            mask[:, lo:hi] = True
            for h in range(Hkv):
                oh, lh = _attend(q[b, h * G:(h + 1) * G].float()[None], k[:, h], v[:, h], mask, scale)
                o[h * G:(h + 1) * G] = oh[0]
                l2[h * G:(h + 1) * G] = lh[0]
        out_part[b, :, npre + split] = o
        lp[b, :, npre + split] = l2
    if out is not None:
        for b, n in nparts.items():
            parts = out_part[b:b + 1, :, :n].clone()
            if pre_part is not None:
                parts[:, :, :npres[b]] = pre_part[b:b + 1, :, :npres[b]].float()
            attn_merge(parts.contiguous(), lp[b:b + 1, :, :n].contiguous(), out[b:b + 1])


def attn_prefill_items(items, q, k_cache, v_cache, block_tables, q_limit, scale, out=None, out_part=None,
                       lse_part=None, alt_part=None, alt_lse=None, alt_tok_off=0):
    """Reference for the work-item prefill / cascade kernel (see ops/csrc/attention.hip, attn_tile.hip); items with
    field 6 set write their partial to alt_part / alt_lse at row token - alt_tok_off."""
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    G = Hq // Hkv
    for it in items.tolist():
        q_start, q_count, bt_row, lo, hi, split = it[:6]
        if q_count <= 0:
            continue
        toks = torch.arange(q_start, q_start + q_count, device=q.device)
        lim = q_limit[toks].long()
        kmax = int(min(hi, int(lim.max()) + 1))
        if kmax <= lo:
            o = torch.zeros(q_count, Hq, D, device=q.device)
            l2 = torch.full((q_count, Hq), float("-inf"), device=q.device)
        else:
            k, v = gather_kv(k_cache, v_cache, block_tables[bt_row], kmax)
            pos = torch.arange(kmax, device=q.device)
            mask = (pos[None] >= lo) & (pos[None] < hi) & (pos[None] <= lim[:, None])
            o = torch.zeros(q_count, Hq, D, device=q.device)
            l2 = torch.zeros(q_count, Hq, device=q.device)
            for h in range(Hkv):
                oh, lh = _attend(q[toks, h * G:(h + 1) * G].float(), k[:, h], v[:, h], mask, scale)
                o[:, h * G:(h + 1) * G] = oh
                l2[:, h * G:(h + 1) * G] = lh
        if split < 0:
            out[toks] = o.to(out.dtype)
        elif it[6] and alt_part is not None:
            rows = toks - alt_tok_off
            alt_part[rows, :, split] = o.to(alt_part.dtype)
            alt_lse.view(alt_part.shape[0], Hq, alt_part.shape[2])[rows, :, split] = l2
        else:
            out_part[toks, :, split] = o.to(out_part.dtype)
            lse_part.view(out_part.shape[0], Hq, out_part.shape[2])[toks, :, split] = l2


def attn_merge(part, lse, out, lse_out=None, pre=None, npre=0):
    rows = out.shape[0]
    p = part[:rows].float()
    if pre is not None and npre:  # bf16 prefix partials in slots [0, npre)
        p = p.clone()
        p[:, :, :npre] = pre[:rows, :, :npre].float()
    l = lse.view(part.shape[0], part.shape[1], part.shape[2])[:rows]
    M = l.amax(-1, keepdim=True)
    Mu = torch.where(torch.isinf(M), torch.zeros_like(M), M)
    f = torch.exp2(l - Mu)
    L = f.sum(-1, keepdim=True)
    pz = torch.where(f[..., None] > 0, p, torch.zeros_like(p))  # unwritten slots (lse -inf) may hold anything
    o = (f[..., None] * pz).sum(2) / torch.where(L > 0, L, torch.ones_like(L))
    out.copy_(o.to(out.dtype))
    if lse_out is not None:
        lse_out.view(rows, -1).copy_(torch.where(L[..., 0] > 0, Mu[..., 0] + torch.log2(L[..., 0]),
                                                 torch.full_like(L[..., 0], float("-inf"))))


def process_logits(logits, proc, mask_tab, counts):
    """The sampler's per-row logits processing (csrc/sampling.hip RowProc) in fp32: penalties from the row's token
    counts, then the grammar bitmask (-inf where a bit is 0). Returns (processed fp32 logits, forced ids or -1)."""
    B, V = logits.shape
    x = logits.float().clone()
    forced = torch.full((B,), -1, dtype=torch.long)
    pr = proc[:B].cpu()
    for b in range(B):
        mode, arg, slot = int(pr[b, 0]), int(pr[b, 1]), int(pr[b, 2])
        pres, freq = pr[b, 3:5].clone().view(torch.float32).tolist()
        if mode == 2:
            forced[b] = arg
            continue
        if slot >= 0:
            c = counts[slot, :V].to(x.device).float()
            x[b] -= freq * c + pres * (c > 0).float()
        if mode == 1:
            words = mask_tab[arg].to(torch.int64) & 0xFFFFFFFF
            bits = (words[:, None] >> torch.arange(32)) & 1
            keep = bits.reshape(-1)[:V].bool().to(x.device)
            x[b].masked_fill_(~keep, float("-inf"))
    return x, forced


def sample(logits, temperature=None, top_p=None, top_k=None, seeds=None, step=None, out=None, proc=None,
           mask_tab=None, counts=None):
    """CPU sampler with the same semantics (not the same random stream) as the HIP kernel."""
    B, V = logits.shape
    forced = None
    if proc is not None:
        x, forced = process_logits(logits, proc, mask_tab, counts)
    else:
        x = logits.float()
    res = torch.empty(B, dtype=torch.long, device=logits.device)
    for b in range(B):
        if forced is not None and int(forced[b]) >= 0:
            res[b] = int(forced[b])
            continue
        t = float(temperature[b]) if temperature is not None else 0.0
        if not t > 0:
            res[b] = int(torch.argmax(x[b]))
            continue
        z = x[b] / t
        p = torch.softmax(z, -1)
        tp = float(top_p[b]) if top_p is not None else 1.0
        tk = int(top_k[b]) if top_k is not None else 0
        order = torch.argsort(p, descending=True)
        ps = p[order]
        keep = torch.ones(V, dtype=torch.bool, device=p.device)
        if tk > 0:
            keep[tk:] = False
        if tp < 1.0:
            above = torch.cumsum(ps, 0) - ps
            keep &= above < tp
        ps = torch.where(keep, ps, torch.zeros_like(ps))
        gen = torch.Generator(device="cpu")
        seed = int(seeds[b]) if seeds is not None else 0x1234
        stepv = int(step[0]) if step is not None else 0
        gen.manual_seed((seed * 1000003 + stepv) & 0x7FFFFFFFFFFFFFFF)
        idx = torch.multinomial(ps.cpu() / ps.sum().cpu(), 1, generator=gen)
        res[b] = order[idx.to(order.device)]
    if proc is not None and counts is not None:
        for b in range(B):
            slot = int(proc[b, 2])
            if slot >= 0:
                counts[slot, int(res[b])] += 1
    if out is not None:
        out[:B].copy_(res)
        return out
    return res


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, D] fp32 table: cos of the D/2 frequencies then sin (rotate-half / NeoX convention).

    ``scaling`` follows the HF ``rope_scaling`` dict: ``{"rope_type": "llama3", "factor", "low_freq_factor",
    "high_freq_factor", "original_max_position_embeddings"}`` or ``{"rope_type": "linear", "factor"}``.
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling:
        kind = scaling.get("rope_type", scaling.get("type"))
        if kind == "llama3":
            factor = scaling["factor"]
            lf, hf = scaling["low_freq_factor"], scaling["high_freq_factor"]
            old = scaling["original_max_position_embeddings"]
            low_wl, high_wl = old / lf, old / hf
            wl = 2 * math.pi / inv
            smooth = (old / wl - lf) / (hf - lf)
            scaled = torch.where(wl > low_wl, inv / factor, inv)
            mid = (wl <= low_wl) & (wl >= high_wl)
            inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        elif kind == "linear":
            inv = inv / scaling["factor"]
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def moe_route(logits: torch.Tensor, k: int, bm: int = 64):
    """fp32 reference of csrc/moe.hip moe_route: (topk_w, topk_e, perm_tok, perm_w, expert_off, tile_off)."""
    T, E = logits.shape
    p = torch.softmax(logits.float(), dim=-1)
    # descending by probability, lowest expert index first on ties (the kernel's order)
    order = torch.argsort(-p + torch.arange(E, device=p.device) * 1e-12, dim=-1, stable=True)[:, :k]
    w = torch.gather(p, 1, order)
    w = w / w.sum(-1, keepdim=True)
    te = order.to(torch.int32)
    flat = te.reshape(-1).long()
    perm = torch.argsort(flat, stable=True)
    counts = torch.bincount(flat, minlength=E)
    eo = torch.zeros(E + 1, dtype=torch.int32, device=p.device)
    eo[1:] = torch.cumsum(counts, 0)
    to = torch.zeros(E + 1, dtype=torch.int32, device=p.device)
    to[1:] = torch.cumsum((counts + bm - 1) // bm, 0)
    return w.float(), te, (perm // k).to(torch.int32), w.reshape(-1)[perm].float(), eo, to


def grouped_gemm(x, w, perm_tok, perm_w, expert_off, e_lo, gather, y, out):
    e_n = w.shape[0]
    eo = expert_off.tolist()
    for j in range(e_n):
        a, b = eo[e_lo + j], eo[e_lo + j + 1]
        if a == b:
            continue
        rows = x[perm_tok[a:b].long()] if gather else x[a:b]
        yy = rows.float() @ w[j].float().t()
        if out is not None:
            out.index_add_(0, perm_tok[a:b].long(), yy * perm_w[a:b, None])
        else:
            y[a:b] = yy.to(y.dtype)


# ---- expert-parallel all-to-all (csrc/moe.hip ep_*): CPU references of the same image layout -------------------
def _ep_meta(img: torch.Tensor, q: int, C: int) -> torch.Tensor:
    """int32 view of destination block q's metadata rows: [count, 0, 0, 0, expert of slot 0 .. C-1, ...]."""
    return img[q, C:].reshape(-1).view(torch.int32)


def ep_dispatch(x, topk_e, lo, n_own, El, C, img, slot_map):
    ep = img.shape[0]
    k = topk_e.shape[1]
    te = topk_e[lo:lo + n_own].reshape(-1).long()
    counts = [0] * ep
    for i, e in enumerate(te.tolist()):
        q = e // El
        pos = counts[q]
        counts[q] += 1
        slot_map[i] = q * img.shape[1] + pos
        _ep_meta(img, q, C)[4 + pos] = e - q * El
        img[q, pos] = x[lo + i // k]
    for q in range(ep):
        m = _ep_meta(img, q, C)
        m[0:4] = torch.tensor([counts[q], 0, 0, 0], dtype=torch.int32)
        m[4 + counts[q]:4 + C] = -1


def ep_recv_route(img, C, El, bm):
    ep, rows = img.shape[0], img.shape[1]
    ents = []  # (expert, row) of every valid slot, in (source, slot) order
    for p in range(ep):
        m = _ep_meta(img, p, C)
        n = int(m[0])
        for s in range(n):
            ents.append((int(m[4 + s]), p * rows + s))
    S = ep * C
    perm_tok = torch.zeros(S, dtype=torch.int32)
    perm_w = torch.zeros(S, dtype=torch.float32)
    eo = torch.zeros(El + 1, dtype=torch.int32)
    to = torch.zeros(El + 1, dtype=torch.int32)
    pos = 0
    for e in range(El):
        seg = [r for ex, r in ents if ex == e]
        perm_tok[pos:pos + len(seg)] = torch.tensor(seg, dtype=torch.int32)
        perm_w[pos:pos + len(seg)] = 1.0
        pos += len(seg)
        eo[e + 1] = pos
        to[e + 1] = to[e] + (len(seg) + bm - 1) // bm
    return perm_tok, perm_w, eo, to


def ep_combine(back, slot_map, topk_w, lo, n_own, out):
    k = topk_w.shape[1]
    for i in range(n_own):
        acc = torch.zeros(back.shape[-1], dtype=torch.float32)
        for j in range(k):
            acc += float(topk_w[lo + i, j]) * back[int(slot_map[i * k + j])].float()
        out[i] = acc.to(out.dtype)
