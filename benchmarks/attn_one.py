"""Single attention case for PMC-counter profiling (rocprofv3 --pmc): cascade prefix pass, chunk 576
(``attn_one.py [variant] [chunk]``), or a causal prefill of T tokens as the engine plans it
(``attn_one.py causal T [variant]``)."""
import math
import sys

import torch

from kafka_llm_service_amd import ops

if len(sys.argv) > 2 and sys.argv[1] == "causal":
    from kafka_llm_service_amd.engine.model_runner import plan_prefill_items

    dev = torch.device("cuda:0")
    Hq, Hkv, D, T = 32, 8, 128, int(sys.argv[2])
    cvar = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    k = torch.randn(T // 16 + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(T // 16 + 8, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
    bt = torch.arange(T // 16 + 4, dtype=torch.int32, device=dev)[None].contiguous()
    q = torch.randn(T, Hq, D, device=dev, dtype=torch.bfloat16)
    ql = torch.arange(T, dtype=torch.int32, device=dev)
    tile = ops.tile_rows(cvar) // (Hq // Hkv)
    tiles = [(t0, min(tile, T - t0), 0, t0 + min(tile, T - t0), T) for t0 in range(0, T, tile)]
    items, splits, ranges = plan_prefill_items(tiles, Hkv, 256, 256)
    it = torch.tensor(items, dtype=torch.int32, device=dev)
    o = torch.empty(T, Hq, D, device=dev, dtype=torch.bfloat16)
    part = torch.empty(T, Hq, max(1, splits), D, device=dev)
    lse = torch.full((T, Hq, max(1, splits)), float("-inf"), device=dev)
    for _ in range(10):
        ops.attn_prefill(it, q, k, v, bt, ql, D ** -0.5, out=o, out_part=part, lse_part=lse, variant=cvar)
        for lo, hi in ranges:
            ops.attn_merge(part[lo:hi], lse[lo:hi], o[lo:hi])
    torch.cuda.synchronize()
    print("done")
    sys.exit(0)
variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 576
dev = torch.device("cuda:0")
Hq, Hkv, D, B, P = 32, 8, 128, 64, 18000
G = Hq // Hkv
n_pref = P // 16
k = torch.randn(n_pref + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
v = torch.randn(n_pref + 8, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
bt = torch.arange(n_pref + 4, dtype=torch.int32, device=dev)[None].repeat(B, 1).contiguous()
q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
ql = torch.full((B,), P + 10, dtype=torch.int32, device=dev)
tile = ops.tile_rows(variant) // G
nc = math.ceil(P / chunk)
items = torch.tensor([(g0, min(tile, B - g0), 0, c * chunk, min(P, (c + 1) * chunk), c, 0, 0)
                      for g0 in range(0, B, tile) for c in range(nc)], dtype=torch.int32, device=dev)
part = torch.empty(B, Hq, nc, D, device=dev)
lse = torch.empty(B, Hq, nc, device=dev)
for _ in range(10):
    ops.attn_prefill(items, q, k, v, bt, ql, D ** -0.5, out_part=part, lse_part=lse, variant=variant)
torch.cuda.synchronize()
print("done")
