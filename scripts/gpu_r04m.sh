#!/bin/bash
# Round 4 pass M: decode work-item target (workgroup waves) and the BLAS library of the mixed-step gate_up.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/bench_m.jsonl
for round in 1 2; do
for cfg in "KAFKA_X=base" "KAFKA_DECODE_TARGET=768" "KAFKA_DECODE_TARGET=1536" "KAFKA_DECODE_TARGET=2304" "TORCH_BLAS_PREFER_HIPBLASLT=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_m.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c100-175)"
done
done
