#!/bin/bash
# Served burst TTFT vs the prefill cost budget (KAFKA_PREFILL_COST_BUDGET; default 512)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/serve
for b in ${BUDGETS:-256 384 512}; do
  KAFKA_PREFILL_COST_BUDGET=$b timeout -k 10 450 python benchmarks/serve_bench.py --backend engine --model llama3-8b \
    --threads 64 --turns 4 --max-tokens 128 > gpurun_out/serve/burst_budget_$b.log 2>&1 || { tail -30 gpurun_out/serve/burst_budget_$b.log; exit 1; }
  tail -1 gpurun_out/serve/burst_budget_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['ttft_p50_ms'], d['ttft_p99_ms'], d['output_tok_s'], {k: v[0] for k, v in d['ttft_p50_p99_ms_by_turn'].items()})"
done
