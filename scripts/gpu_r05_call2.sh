#!/bin/bash
# host/GPU timeline of the headline (kernel trace + roctx host spans), eager and hipGraph, then the A/B pairs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for mode in eager graphs; do
  extra=""; [[ $mode == graphs ]] && extra="--graphs"
  cd /tmp && KAFKA_ROCTX=1 PYTHONPATH=$R timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace -d "$R/gpurun_out/tl_$mode" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 $extra > "$R/gpurun_out/tl_$mode.log" 2>&1 || { tail -30 "$R/gpurun_out/tl_$mode.log"; exit 1; }
  tail -1 "$R/gpurun_out/tl_$mode.log" | cut -c1-200
  cd "$R"
done
AB_PAIRS=${AB_PAIRS:-2} AB_SEQ="${AB_SEQ:-new old newg}" bash scripts/gpu_r05_ab.sh
