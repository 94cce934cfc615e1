#!/bin/bash
# HTTP serving TTFT breakdown on one GPU: burst (all threads start together) and staggered arrivals, traced.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mode in ${MODES:-burst stagger}; do
  extra=""; [[ $mode == stagger ]] && extra="--stagger ${STAGGER:-2}"
  rm -f /tmp/ktr.*
  echo "== serve $mode $(date +%T)"
  KAFKA_TRACE_FILE=/tmp/ktr timeout -k 10 400 python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads 64 --turns 4 --max-tokens 128 $extra $SERVE_EXTRA > gpurun_out/serve_$mode.log 2>&1
  rc=$?
  if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/serve_$mode.log; then echo "GPU fault"; exit 3; fi
  [[ $rc == 0 ]] || { echo "serve failed rc=$rc"; tail -30 gpurun_out/serve_$mode.log; exit 1; }
  tail -1 gpurun_out/serve_$mode.log
  python scripts/ttft_breakdown.py "/tmp/ktr.*.json" | tee gpurun_out/ttft_breakdown_$mode.txt
done
