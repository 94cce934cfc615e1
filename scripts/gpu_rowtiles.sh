#!/bin/bash
# Streaming GEMM beyond 128 rows (row tiles): kernel tests, microbench vs hipBLASLt, bench A/B (STREAM_MAX_M 128/256).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "wstream" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rowtiles.log 2>&1 || { tail -40 gpurun_out/t_rowtiles.log; exit 1; }
tail -1 gpurun_out/t_rowtiles.log
timeout -k 10 400 python benchmarks/stream_split_bench.py > gpurun_out/stream_rowtiles.log 2>&1 || { tail -20 gpurun_out/stream_rowtiles.log; exit 1; }
grep gemm gpurun_out/stream_rowtiles.log
KAFKA_STREAM_MAX_M=256 timeout -k 10 600 python -u -m pytest tests -m gpu -k "engine or smoke" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rowtiles_engine.log 2>&1 || { tail -40 gpurun_out/t_rowtiles_engine.log; exit 1; }
tail -1 gpurun_out/t_rowtiles_engine.log
ARMS="KAFKA_STREAM_MAX_M=128;KAFKA_STREAM_MAX_M=256" ROUNDS=2 STEPS=200 WARM=20 bash scripts/gpu_ab_env.sh
