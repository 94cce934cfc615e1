#!/usr/bin/env python3
"""Per-phase shader-clock anatomy of the tile attention kernel's interior loop (diagnostic build KAFKA_TILE_ABL=9:
outputs are NOT computed; the stamps are written over out_part). Cascade shape, keys per workgroup from argv."""
import os
import sys

import torch

from kafka_llm_service_amd import ops

assert os.environ.get("KAFKA_TILE_ABL") == "9"
dev = torch.device("cuda:0")
Hq, Hkv, D, B = 32, 8, 128, 64
G = Hq // Hkv
P = 18048
nk = int(sys.argv[1]) if len(sys.argv) > 1 else 576
S = min(32, P // nk)
k = torch.randn(P // 16 + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
v = torch.randn(P // 16 + 8, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
bt = torch.arange(P // 16 + 4, dtype=torch.int32, device=dev).view(1, -1)
q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
ql = torch.full((B,), 1 << 30, dtype=torch.int32, device=dev)
part = torch.zeros(B, Hq, 32, D, device=dev)
lse = torch.empty(B, Hq, 32, device=dev)
tile = 256 // G
items = torch.tensor([(g0, min(tile, B - g0), 0, c * nk, (c + 1) * nk, c, 0, 0) for g0 in range(0, B, tile)
                      for c in range(S)], dtype=torch.int32, device=dev)
for _ in range(5):
    ops.attn_prefill(items, q, k, v, bt, ql, 0.088, out_part=part, lse_part=lse, variant=3)
torch.cuda.synchronize()
st = part.view(-1).view(torch.int64)[: items.shape[0] * Hkv * 4 * 8].view(-1, 8).cpu().double()
tiles = st[:, 4].clamp(min=1)
per = st[:, :4] / tiles[:, None]
names = ["wait+barrier", "dma issue", "QK^T+max", "rescale+exp+PV"]
print(f"keys/wg {nk}  waves {st.shape[0]}  interior tiles/wave {tiles.mean():.1f}")
for i, n in enumerate(names):
    col = per[:, i]
    print(f"  {n:16s} cycles/tile: median {col.median():7.0f}  p10 {col.quantile(0.1):7.0f}  p90 {col.quantile(0.9):7.0f}")
print(f"  total            cycles/tile: median {per.sum(1).median():7.0f}")
