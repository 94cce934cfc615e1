#!/bin/bash
# Round 4 pass F: (1) any-order launch probe (does a same-stream successor start before its predecessor ends on
# gfx950?), (2) tile-kernel workgroup phase stamps on the cascade shape, (3) headline vs --tool-frac 0.25 after the
# plan-ahead predicate fix, (4) the 18k synthetic shared prefix through the HTTP API.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 ./build_probe/anyorder_probe > gpurun_out/anyorder_probe.jsonl 2>&1 || { cat gpurun_out/anyorder_probe.jsonl; exit 1; }
cat gpurun_out/anyorder_probe.jsonl
timeout -k 10 120 python -u benchmarks/attn_tile_stamps.py > gpurun_out/tile_stamps.jsonl 2>&1 || { tail -20 gpurun_out/tile_stamps.jsonl; exit 1; }
cat gpurun_out/tile_stamps.jsonl
: > gpurun_out/bench_tool_f.jsonl
for v in base tool25 base tool25; do
  case $v in base) A="";; tool25) A="--tool-frac 0.25";; esac
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 $A > gpurun_out/bench_f_$v.log 2>&1 || { tail -20 gpurun_out/bench_f_$v.log; exit 1; }
  tail -1 gpurun_out/bench_f_$v.log >> gpurun_out/bench_tool_f.jsonl
  tail -1 gpurun_out/bench_f_$v.log | cut -c1-140
done
echo "== serve sys18k $(date +%T)"
timeout -k 10 400 python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 \
  --max-tokens 128 --stagger 2 --system-tokens 18000 > gpurun_out/serve_sys18k.log 2>&1 || { tail -30 gpurun_out/serve_sys18k.log; exit 1; }
tail -1 gpurun_out/serve_sys18k.log
