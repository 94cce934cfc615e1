"""Where does the MT=4 grouped kernel differ from the fp32 reference (debug helper, GPU)."""
import torch
from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import reference as ref

dev = torch.device("cuda:0")
for (T, d, F, E, e_lo, e_n) in [(200, 512, 1024, 8, 2, 4), (256, 512, 1024, 8, 0, 8), (300, 1024, 512, 8, 0, 8),
                                (200, 4096, 1792, 8, 0, 8)]:
    torch.manual_seed(9)
    x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    w13 = (torch.randn(e_n, 2 * F, d, device=dev) * d ** -0.5).to(torch.bfloat16)
    r = ops.moe_route(torch.randn(T, E, device=dev).to(torch.bfloat16), 2)
    rc = ops.MoERouting(*(t.cpu() for t in (r.topk_w, r.topk_e, r.perm_tok, r.perm_w, r.expert_off, r.tile_off)), E)
    w13t = ops.tile_experts(w13, glu=True)
    a = ops.grouped_stream_glu(x, w13t, r, e_lo=e_lo).float().cpu()
    h_ref = torch.zeros(T * 2, 2 * F)
    ref.grouped_gemm(x.cpu().float(), w13.cpu().float(), rc.perm_tok, rc.perm_w, rc.expert_off, e_lo, True, h_ref, None)
    eo = rc.expert_off.tolist()
    y = ref.silu_mul(h_ref).float()
    for e in range(e_lo, e_lo + e_n):
        lo, hi = eo[e], eo[e + 1]
        if hi <= lo:
            continue
        err = (a[lo:hi] - y[lo:hi]).abs()
        bad = (err > 0.05).nonzero()
        rows = sorted(set(bad[:, 0].tolist()))
        cols = sorted(set(bad[:, 1].tolist()))
        print(f"T={T} d={d} F={F} e={e} rows={hi - lo} max_err={err.max():.3f} bad_rows={rows[:12]}.. n={len(rows)} "
              f"bad_cols={cols[:8]}.. n={len(cols)}", flush=True)
