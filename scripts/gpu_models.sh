#!/bin/bash
# Other model families on one MI355X (not the headline): MoE layer microbench, Mixtral-8x7B serving bench (128 threads,
# BASELINE config 5 shape), Llama-3-70B on ONE GPU (140 GB of bf16 weights in 288 GB of HBM). Stops at the first
# failure or GPU fault. Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_models.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/$name.log; then echo "GPU fault in $name"; exit 3; fi
  [[ $rc == 0 ]] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }
  grep -v "Warn\|amdgpu.ids" gpurun_out/$name.log | tail -${TAILN:-1} | cut -c1-400
}
TAILN=8 run moe_bench 300 python benchmarks/moe_bench.py
run bench_mixtral 400 python bench.py --model mixtral-8x7b --threads 128 --steps 60 --warmup 20
run bench_70b_tp1 500 python bench.py --model llama3-70b --threads 64 --steps 40 --warmup 10
echo "== done $(date +%T)"
