#!/bin/bash
# Round 4 pass X: gate_up of 129..256-row (mixed) steps on the streaming kernel (two XCD-shared 128-row tiles,
# fused SwiGLU) instead of hipBLASLt + silu_mul — microbench, then bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 200 --shapes 8b.gate_up,8b.qkv,8b.o,8b.down > gpurun_out/wsb_x200.log 2>&1 || { tail -20 gpurun_out/wsb_x200.log; exit 1; }
timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 160 --shapes 8b.gate_up > gpurun_out/wsb_x160.log 2>&1 || { tail -20 gpurun_out/wsb_x160.log; exit 1; }
tail -4 gpurun_out/wsb_x200.log; tail -1 gpurun_out/wsb_x160.log
: > gpurun_out/bench_x.jsonl
for round in 1 2; do
for cfg in "KAFKA_STREAM_GU_MAX_M=0" "KAFKA_STREAM_GU_MAX_M=256"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_x.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
