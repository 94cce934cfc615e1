#!/usr/bin/env python3
"""Cascade tile-kernel cost model: at a FIXED grid (32 key chunks x 8 KV heads = 256 workgroups, 64 decode rows x
4 heads per workgroup) vary the shared prefix length, so per-workgroup time t(n) = a + b n separates the fixed
per-workgroup cost a (launch, Q / page-table loads, pipeline fill, partial write-out) from the per-32-key-block cost b."""
import json
import math
import os
import statistics

import torch

from kafka_llm_service_amd import ops

dev = torch.device("cuda:0")
Hq, Hkv, D, B = 32, 8, 128, 64
G = Hq // Hkv
for P in [int(x) for x in os.environ.get("PREFIXES", "4608,9216,18432,36864,73728").split(",")]:
    nc = 32
    chunk = P // nc
    n_pref = P // 16
    k = torch.randn(n_pref + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    v = torch.randn(n_pref + 8, Hkv, D, 16, device=dev, dtype=torch.bfloat16)
    bt = torch.arange(n_pref + 4, dtype=torch.int32, device=dev)[None].repeat(B, 1).contiguous()
    q = torch.randn(B, Hq, D, device=dev, dtype=torch.bfloat16)
    ql = torch.full((B,), P + 10, dtype=torch.int32, device=dev)
    items = torch.tensor([(0, B, 0, c * chunk, (c + 1) * chunk, c, 0, 0) for c in range(nc)], dtype=torch.int32,
                         device=dev)
    part = torch.empty(B, Hq, nc, D, device=dev)
    lse = torch.empty(B, Hq, nc, device=dev)

    ref_part, ref_lse = None, None
    for variant in [int(x) for x in os.environ.get("VARIANTS", "0").split(",")]:
      def run():
        ops.attn_prefill(items, q, k, v, bt, ql, D ** -0.5, out_part=part, lse_part=lse, variant=variant)

      ts = []
      for _ in range(5):
          run()
          torch.cuda.synchronize()
          s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
          s.record()
          for _ in range(20):
              run()
          e.record()
          torch.cuda.synchronize()
          ts.append(s.elapsed_time(e) * 1e3 / 20)
      us = statistics.median(ts)
      if ref_part is None:
          ref_part, ref_lse = part.clone(), lse.clone()
          err = 0.0
      else:
          err = max((part - ref_part).abs().max().item(), (lse - ref_lse).abs().max().item())
      flops = 4 * B * Hq * P * D
      print(json.dumps({"prefix": P, "blocks_per_wg": chunk // 32, "us": round(us, 1),
                        "TF/s": round(flops / us / 1e6, 1), "variant": variant, "max_err": err}), flush=True)
    del k, v
