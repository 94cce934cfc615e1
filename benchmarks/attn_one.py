"""Single attention case for PMC-counter profiling (rocprofv3 --pmc): cascade prefix pass, chunk 576."""
import math
import sys

import torch

from kafka_llm_service_amd import ops

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
