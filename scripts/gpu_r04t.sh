#!/bin/bash
# Round 4 pass T: three-row-tile decode GEMM for 65..96 rows — kernel tests, then bench A/B vs the four-tile plan.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream or engine or cascade or early or graph" > gpurun_out/t_t.log 2>&1 || { tail -40 gpurun_out/t_t.log; exit 1; }
tail -1 gpurun_out/t_t.log
: > gpurun_out/bench_t.jsonl
for round in 1 2 3; do
for cfg in "KAFKA_WSTREAM_MT3=1" "KAFKA_WSTREAM_MT3=0"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_t.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c100-175)"
done
done
