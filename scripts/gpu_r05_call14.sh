#!/bin/bash
# staggered tile loop (waves 4-7 half a tile behind, KAFKA_TILE_STAGGER=1): tile numerics under it, cascade launch
# alone both ways, headline A/B (new = plain, newe = staggered)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_TILE_STAGGER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn" > gpurun_out/call14_tests.log 2>&1 || { tail -30 gpurun_out/call14_tests.log; exit 1; }
echo "stagger $(tail -1 gpurun_out/call14_tests.log)"
for st in 0 1; do
  KAFKA_TILE_STAGGER=$st timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_stagger_$st.jsonl 2>&1 || { tail -20 gpurun_out/cascade_stagger_$st.jsonl; exit 1; }
  echo "stagger=$st $(grep -E '"cascade"' gpurun_out/cascade_stagger_$st.jsonl | cut -c1-40)"
done
AB_PAIRS=3 AB_SEQ="new newe" AB_ENV="KAFKA_TILE_STAGGER=1" bash scripts/gpu_r05_ab.sh
