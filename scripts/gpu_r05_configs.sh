#!/bin/bash
# BASELINE configs 4 and 5 at real size on one MI355X: Mixtral-8x7B at 128 threads (bench.py) and Llama-3-70B
# (tiled-only, TP = 1) through /v1/threads/{id}/agent/run with the served ~18k-token system prompt and the tool chain.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
if [[ -z $SKIP_MIXTRAL ]]; then
  timeout -k 10 900 python bench.py --model mixtral-8x7b --threads 128 --steps ${MX_STEPS:-150} --warmup 20 > gpurun_out/mixtral_128.log 2>&1 || { tail -30 gpurun_out/mixtral_128.log; exit 1; }
  tail -1 gpurun_out/mixtral_128.log | cut -c1-300
fi
if [[ -z $SKIP_70B ]]; then
  timeout -k 10 1000 python scripts/config4_real.py --out gpurun_out/config4_real > gpurun_out/config4_real.log 2>&1 || { tail -40 gpurun_out/config4_real.log; exit 1; }
  tail -1 gpurun_out/config4_real.log | cut -c1-1500
fi
