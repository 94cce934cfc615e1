#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/kt.log 2>&1 || { tail -30 gpurun_out/kt.log; exit 1; }
tail -2 gpurun_out/kt.log
timeout -k 10 600 python benchmarks/attn_bench.py ${ATTN_ARGS} > gpurun_out/attn_bench.log 2>&1 || { tail -30 gpurun_out/attn_bench.log; exit 1; }
cat gpurun_out/attn_bench.log
