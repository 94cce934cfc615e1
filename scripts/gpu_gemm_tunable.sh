#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=100
timeout -k 10 900 python benchmarks/gemm_bench.py 64 --libs-only > gpurun_out/gemm_bench_tunable.log 2>&1 || { tail -30 gpurun_out/gemm_bench_tunable.log; exit 1; }
grep gemm gpurun_out/gemm_bench_tunable.log
ls gpurun_out/
