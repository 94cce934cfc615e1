#!/bin/bash
# Round 4 pass J: gates v2 (arrival tree + per-XCD done flags: no hot line) — equality test, then bench modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "early" > gpurun_out/t_early.log 2>&1 || { tail -60 gpurun_out/t_early.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_early.log | tail -2
for cfg in "KAFKA_EARLY=0" "KAFKA_EARLY=1 KAFKA_GATE_MODE=0" "KAFKA_EARLY=1 KAFKA_GATE_MODE=1" "KAFKA_EARLY=1 KAFKA_GATE_MODE=3" "KAFKA_EARLY=1 KAFKA_GATE_MODE=2"; do
  env $cfg timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c1-150)"
done
for w in 8 4; do
  KAFKA_TILE_WAVES=$w timeout -k 10 200 python -u benchmarks/attn_tile_anatomy.py --variants 3 --keys 576 2>&1 | grep keys_per | sed "s/^/waves$w /" || exit 1
done
KAFKA_TILE_WAVES=4 timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
echo "KAFKA_TILE_WAVES=4 $(tail -1 gpurun_out/bench_cfg.log | cut -c1-150)"
