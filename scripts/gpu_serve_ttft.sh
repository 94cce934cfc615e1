#!/bin/bash
# HTTP serving TTFT breakdown on one GPU: burst (all threads start together) and staggered arrivals, traced, for
# each served prompt (PROMPTS="reference compact": the reference's 13 sections ~37k tokens / our compact ~20k).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for prompt in ${PROMPTS:-reference}; do
for mode in ${MODES:-burst stagger}; do
  extra=""; [[ $mode == stagger ]] && extra="--stagger ${STAGGER:-2}"
  rm -f /tmp/ktr.*
  tag=${mode}_${prompt}
  echo "== serve $tag $(date +%T)"
  KAFKA_PROMPT=$prompt KAFKA_TRACE_FILE=/tmp/ktr timeout -k 10 400 python benchmarks/serve_bench.py --backend engine \
    --model llama3-8b --threads 64 --turns 4 --max-tokens 128 $extra $SERVE_EXTRA > gpurun_out/serve_$tag.log 2>&1
  rc=$?
  if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/serve_$tag.log; then echo "GPU fault"; exit 3; fi
  [[ $rc == 0 ]] || { echo "serve failed rc=$rc"; tail -30 gpurun_out/serve_$tag.log; exit 1; }
  tail -1 gpurun_out/serve_$tag.log
  python scripts/ttft_breakdown.py "/tmp/ktr.*.json" | tee gpurun_out/ttft_breakdown_$tag.txt
  if [[ -n "$KEEP_TRACES" ]]; then mkdir -p gpurun_out/traces_$tag && cp /tmp/ktr.*.json gpurun_out/traces_$tag/; fi
done
done
exit 0
