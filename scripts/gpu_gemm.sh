#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python benchmarks/gemm_bench.py ${GEMM_MS:-1,32,64} > gpurun_out/gemm_bench.log 2>&1 || { tail -30 gpurun_out/gemm_bench.log; exit 1; }
grep gemm gpurun_out/gemm_bench.log
