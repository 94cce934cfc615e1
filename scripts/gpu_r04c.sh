#!/bin/bash
# Round 4: HTTP TTFT with the Llama-3-class tokenizer (reference prompt ~18.2k tokens): burst + staggered, plus the
# headline's 18k synthetic shared prefix through the API (the API-path tax on the engine metric).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
MODES="burst stagger" bash scripts/gpu_serve_ttft.sh || exit 1
echo "== serve sys18k $(date +%T)"
timeout -k 10 400 python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 \
  --max-tokens 128 --stagger 2 --system-tokens 18000 > gpurun_out/serve_sys18k.log 2>&1 || { tail -30 gpurun_out/serve_sys18k.log; exit 1; }
tail -1 gpurun_out/serve_sys18k.log
