"""lm_head (128256 x 4096) at 64 rows: one 64-row tile vs two 32-row tiles sharing each weight slice on one XCD."""
import json, torch, sys
sys.path.insert(0, "benchmarks")
from kafka_llm_service_amd import ops
from kafka_llm_service_amd.ops import _ext
from wstream_bench import timeit
ext = _ext.load()
dev = torch.device("cuda:0")
N, K = 128256, 4096
wts = [ops.tile_weight((torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)) for _ in range(2)]
x = torch.randn(64, K, device=dev, dtype=torch.bfloat16)
y = torch.empty(64, N, device=dev, dtype=torch.bfloat16)
for mt, kc, kw, pin in [(2, 256, 2, 1), (2, 256, 2, 0), (1, 256, 1, 0), (1, 256, 1, 1), (1, 256, 2, 0), (1, 256, 2, 1)]:
    t = timeit([lambda wt=wt: ext.wstream_gemm_cfg(x, wt, y, None, mt, kc, 1, True, kw, pin) for wt in wts])
    print(json.dumps({"mt": mt, "kw": kw, "pin": pin, "us": round(t, 1)}), flush=True)
