#!/bin/bash
# Round 4 pass Z: suffix decode with an L2 prefetch of each wave's next K/V block (KAFKA_DECODE_OCC3=2: two LDS-DMA
# dword touches per lane, no VGPRs) — numerics under the switch, then bench A/B against the default (OCC3=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_DECODE_OCC3=2 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn_decode or engine_matches or cascade" > gpurun_out/t_z.log 2>&1 || { tail -40 gpurun_out/t_z.log; exit 1; }
tail -1 gpurun_out/t_z.log
: > gpurun_out/bench_z.jsonl
for round in 1 2; do
for cfg in "KAFKA_DECODE_OCC3=1" "KAFKA_DECODE_OCC3=2"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_z.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
