#!/bin/bash
# cascade ring of 4 slots (3 tiles in flight) vs 3: tile tests, cascade launch alone, headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_TILE_NSLOT=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn" > gpurun_out/call10_tests.log 2>&1 || { tail -30 gpurun_out/call10_tests.log; exit 1; }
echo "nslot4 $(tail -1 gpurun_out/call10_tests.log)"
for n in 3 4; do
  KAFKA_TILE_NSLOT=$n timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_nslot_$n.jsonl 2>&1 || { tail -20 gpurun_out/cascade_nslot_$n.jsonl; exit 1; }
  echo "nslot=$n $(grep -E '"cascade"' gpurun_out/cascade_nslot_$n.jsonl | cut -c1-40)"
done
AB_PAIRS=2 AB_SEQ="new newe" AB_ENV="KAFKA_TILE_NSLOT=4" bash scripts/gpu_r05_ab.sh
