#!/bin/bash
# half-pipelined tile body (KAFKA_TILE_PIPE=1) vs the plain one, both on the raw v_exp_f32: tile tests under each,
# cascade launch alone, then the headline A/B (new = PIPE 0, newe = PIPE 1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for p in 0 1; do
  KAFKA_TILE_PIPE=$p timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attn" > gpurun_out/call9_tests_$p.log 2>&1 || { tail -30 gpurun_out/call9_tests_$p.log; exit 1; }
  echo "pipe=$p $(tail -1 gpurun_out/call9_tests_$p.log)"
  KAFKA_TILE_PIPE=$p timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_pipe_$p.jsonl 2>&1 || { tail -20 gpurun_out/cascade_pipe_$p.jsonl; exit 1; }
  grep -E '"(seq|cascade|decode_fused)"' gpurun_out/cascade_pipe_$p.jsonl | cut -c1-40
done
AB_PAIRS=2 AB_SEQ="new newe" AB_ENV="KAFKA_TILE_PIPE=1" bash scripts/gpu_r05_ab.sh
