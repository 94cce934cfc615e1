#!/bin/bash
# HTTP burst serving with the API event loop under cProfile (KAFKA_API_PROFILE) and the trace breakdown
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f /tmp/ktr.*
KAFKA_API_PROFILE=$GRAFT_REPO_ROOT/gpurun_out/api_profile.txt KAFKA_TRACE_FILE=/tmp/ktr timeout -k 10 400 \
  python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 --max-tokens 128 \
  $SERVE_EXTRA > gpurun_out/serve_prof.log 2>&1 || { tail -30 gpurun_out/serve_prof.log; exit 1; }
tail -1 gpurun_out/serve_prof.log
python scripts/ttft_breakdown.py "/tmp/ktr.*.json" | tee gpurun_out/ttft_breakdown_prof.txt
