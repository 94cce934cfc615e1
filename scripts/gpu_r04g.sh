#!/bin/bash
# Round 4 pass G: early-launched decode layers (KAFKA_EARLY, device gates): kernel + engine GPU tests (bitwise
# equality with ordinary launches), then a same-box bench A/B (EARLY 0/1 interleaved) and the tile ring depth 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "early or wstream or rope or attn or decode or norm or engine_matches or cascade" > gpurun_out/t_early.log 2>&1 || { tail -60 gpurun_out/t_early.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_early.log | tail -3
: > gpurun_out/bench_early.jsonl
for v in 0 1 0 1; do
  KAFKA_EARLY=$v timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_early_$v.log 2>&1 || { tail -20 gpurun_out/bench_early_$v.log; exit 1; }
  tail -1 gpurun_out/bench_early_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['early']=$v; print(json.dumps(d))" >> gpurun_out/bench_early.jsonl
  tail -1 gpurun_out/bench_early.jsonl | cut -c1-150
done
for v in 3 4; do
  KAFKA_TILE_SLOTS=$v timeout -k 10 200 python -u benchmarks/attn_tile_anatomy.py --variants 3 --keys 576,1152 2>&1 | grep keys_per | sed "s/^/slots$v /" || exit 1
done
for cfg in "KAFKA_TILE_SLOTS=4 KAFKA_EARLY=1" "KAFKA_CASCADE_WGS=128 KAFKA_EARLY=1" "KAFKA_CASCADE_WGS=192 KAFKA_EARLY=1" "KAFKA_CASCADE_WGS=128 KAFKA_EARLY=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c1-150)"
done
