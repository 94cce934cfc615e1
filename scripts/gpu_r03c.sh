#!/bin/bash
# round 3: attention bench (variants 0 / 3 on every case) + a 400-step bench with the per-step log (stationarity)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/attn_bench.py > gpurun_out/r03c_attn_bench.log 2>&1 &&
KAFKA_BENCH_STEPLOG=gpurun_out/steplog_400.jsonl timeout -k 10 400 python bench.py --steps 400 --warmup 5 \
  > gpurun_out/r03c_bench_400_5.log 2>&1
