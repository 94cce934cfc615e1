#!/bin/bash
# Round 4 pass AF: re-check older decode-attention switches on the current tree (placement: heads-fast vs
# items-fast; three vs two workgroups per CU) — bench A/B, interleaved x2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/bench_af.jsonl
for round in 1 2; do
for cfg in "KAFKA_DECODE_HEADS_FAST=1" "KAFKA_DECODE_HEADS_FAST=0" "KAFKA_DECODE_OCC3=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_af.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
