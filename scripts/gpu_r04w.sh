#!/bin/bash
# Round 4 pass W: suffix decode overlapped with the cascade (KAFKA_ATTN_OVERLAP=1: any-order decode launch,
# write-through hand-off of the cascade partials) — bitwise test, then bench A/B over the cascade's workgroup count.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "overlap or early_launched" > gpurun_out/t_w.log 2>&1 || { tail -40 gpurun_out/t_w.log; exit 1; }
tail -3 gpurun_out/t_w.log
: > gpurun_out/bench_w.jsonl
for round in 1 2; do
for cfg in "KAFKA_ATTN_OVERLAP=0" "KAFKA_ATTN_OVERLAP=1" "KAFKA_ATTN_OVERLAP=1 KAFKA_PREFIX_WGS=128" "KAFKA_ATTN_OVERLAP=1 KAFKA_PREFIX_WGS=64"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_w.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
