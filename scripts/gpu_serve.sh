#!/bin/bash
# Served TTFT through the HTTP API: the reference prompt, burst and staggered (SERVE_MODES), SERVE_THREADS threads x 4
# turns, extra serve_bench arguments in SERVE_ARGS; logs under gpurun_out/serve/
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/serve
for mode in ${SERVE_MODES:-burst stagger}; do
  A=""; [[ $mode == stagger ]] && A="--stagger 2"
  timeout -k 10 450 python benchmarks/serve_bench.py --backend engine --model llama3-8b --threads ${SERVE_THREADS:-64} --turns 4 \
    --max-tokens 128 $A ${SERVE_ARGS} > gpurun_out/serve/serve_$mode.log 2>&1 || { tail -30 gpurun_out/serve/serve_$mode.log; exit 1; }
  tail -1 gpurun_out/serve/serve_$mode.log | cut -c1-400
done
