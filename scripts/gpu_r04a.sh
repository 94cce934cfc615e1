#!/bin/bash
# Round 4, first GPU pass: sampler logits-processing numerics, tile v3 PMC, headline bench + the --tool-frac A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "sample" --timeout 120 --timeout-method thread > gpurun_out/t_sample.log 2>&1 || { tail -40 gpurun_out/t_sample.log; exit 1; }
tail -1 gpurun_out/t_sample.log
mkdir -p gpurun_out/transcripts
KAFKA_TRANSCRIPT_DIR=$GRAFT_REPO_ROOT/gpurun_out/transcripts timeout -k 10 600 python -u -m pytest tests/test_server_gpu.py tests/test_custom_allreduce_gpu.py -x -v -k "config4 or lost_peer or dp_attention" --timeout 300 --timeout-method thread > gpurun_out/t_c4.log 2>&1 || { tail -60 gpurun_out/t_c4.log; exit 1; }
tail -1 gpurun_out/t_c4.log
bash scripts/gpu_pmc_tile3.sh > gpurun_out/pmc_tile3.log 2>&1 || { tail -20 gpurun_out/pmc_tile3.log; exit 1; }
cat gpurun_out/pmc_tile3/summary.txt
cd "$GRAFT_REPO_ROOT"
: > gpurun_out/bench_ab.jsonl
for v in base tool25 base tool25; do
  case $v in base) A="";; tool25) A="--tool-frac 0.25";; esac
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 $A > gpurun_out/bench_$v.log 2>&1 || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/bench_ab.jsonl
  tail -1 gpurun_out/bench_ab.jsonl | cut -c1-200
done
