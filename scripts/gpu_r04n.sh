#!/bin/bash
# Round 4 pass N: burst TTFT vs the scheduler's per-step prefill cost budget (reference prompt, 64 threads at once).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for b in 512 1024 2048 768; do
  KAFKA_PREFILL_COST_BUDGET=$b timeout -k 10 400 python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 \
    --max-tokens 128 > gpurun_out/serve_budget_$b.log 2>&1 || { tail -30 gpurun_out/serve_budget_$b.log; exit 1; }
  echo "budget $b $(tail -1 gpurun_out/serve_budget_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ttft_p50_ms'], d['ttft_p99_ms'], d['output_tok_s'], d['ttft_p50_p99_ms_by_turn'])")"
done
