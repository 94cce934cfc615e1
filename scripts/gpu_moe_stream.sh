#!/bin/bash
# Grouped weight-streaming expert MLP beyond 128 tokens: kernel tests, MoE layer microbench, Mixtral bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "wstream_grouped" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_grouped.log 2>&1 || { tail -40 gpurun_out/t_grouped.log; exit 1; }
tail -1 gpurun_out/t_grouped.log
timeout -k 10 300 python benchmarks/moe_bench.py > gpurun_out/moe_bench.log 2>&1 || { tail -20 gpurun_out/moe_bench.log; exit 1; }
grep '"T"' gpurun_out/moe_bench.log
ARMS="KAFKA_MOE_STREAM_MAX_T=128;KAFKA_MOE_STREAM_MAX_T=320;KAFKA_MOE_STREAM_MAX_T=640" ROUNDS=1 STEPS=60 WARM=20 BENCH_EXTRA="--model mixtral-8x7b --threads 128" bash scripts/gpu_ab_env.sh
