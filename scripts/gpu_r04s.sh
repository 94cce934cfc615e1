#!/bin/bash
# Round 4 pass S: lower decode GEMM split targets (fewer split-K slabs: o / down S = 4, qkv S = 2) vs the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/bench_s.jsonl
for round in 1 2; do
for cfg in "KAFKA_X=base" "KAFKA_WSTREAM_TARGET=128" "KAFKA_WSTREAM_TARGET=96"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_s.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c100-175)"
done
done
