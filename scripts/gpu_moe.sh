#!/bin/bash
# MoE kernels on one MI355X: numerics tests, then the Mixtral-shaped layer microbenchmark (gpurun_out/moe_bench.log).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "moe or grouped" > gpurun_out/moe_tests.log 2>&1 || { echo "moe tests failed"; tail -40 gpurun_out/moe_tests.log; exit 1; }
tail -2 gpurun_out/moe_tests.log
timeout -k 10 300 python benchmarks/moe_bench.py > gpurun_out/moe_bench.log 2>&1 || { echo "moe bench failed"; tail -30 gpurun_out/moe_bench.log; exit 1; }
cat gpurun_out/moe_bench.log | grep -v Warn
