#!/bin/bash
# Round 4 pass AG: gate_up of 129..256-row (mixed) steps on the skinny MFMA GEMM with its fused SwiGLU epilogue
# (KAFKA_SKINNY=qkv,o,down,gate_up) instead of hipBLASLt + silu_mul — numerics, bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_SKINNY=qkv,o,down,gate_up timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "skinny or engine_matches" > gpurun_out/t_ag.log 2>&1 || { tail -40 gpurun_out/t_ag.log; exit 1; }
tail -1 gpurun_out/t_ag.log
: > gpurun_out/bench_ag.jsonl
for round in 1 2; do
for cfg in "KAFKA_SKINNY=qkv,o,down" "KAFKA_SKINNY=qkv,o,down,gate_up"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ag.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
