#!/bin/bash
# Round 4 pass AE: library GEMM kernels of the padded mixed-step sizes loaded at engine start (KAFKA_WARM_SHAPES)
# vs on first use inside the measured window — the driver's 20/5 window, interleaved x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/bench_ae.jsonl
for round in 1 2 3; do
for cfg in "KAFKA_WARM_SHAPES=0" "KAFKA_WARM_SHAPES=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ae.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
