#!/bin/bash
# Round 4 pass AD: XCD-shared row tiles with CACHED weight loads (KAFKA_WSTREAM_TILE_NT=0; non-temporal loads may
# keep the first tile's lines out of L2) — microbench at M = 64 (two 32-row tiles) and M = 200 (two 128-row tiles),
# then bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "KAFKA_WSTREAM_RT1=1" "KAFKA_WSTREAM_RT1=1 KAFKA_WSTREAM_TILE_NT=0"; do
  env $cfg timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 64 --shapes 8b.gate_up,8b.qkv,8b.o,8b.down > gpurun_out/wsb_ad.log 2>&1 || { tail -20 gpurun_out/wsb_ad.log; exit 1; }
  echo "# $cfg"; tail -4 gpurun_out/wsb_ad.log
done
for cfg in "KAFKA_WSTREAM_TILE_NT=1" "KAFKA_WSTREAM_TILE_NT=0"; do
  env $cfg timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 200 --shapes 8b.gate_up,8b.down > gpurun_out/wsb_ad.log 2>&1 || { tail -20 gpurun_out/wsb_ad.log; exit 1; }
  echo "# M=200 $cfg"; tail -2 gpurun_out/wsb_ad.log
done
: > gpurun_out/bench_ad.jsonl
for round in 1 2; do
for cfg in "KAFKA_WSTREAM_TILE_NT=1" "KAFKA_WSTREAM_RT1=1 KAFKA_WSTREAM_TILE_NT=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ad.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
