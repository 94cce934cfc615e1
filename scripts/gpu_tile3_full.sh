#!/bin/bash
# tile attention v3 in the engine: kernel + engine GPU tests, attention microbenchmark (v0 vs v3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t3_tests.log 2>&1 || { tail -40 gpurun_out/t3_tests.log; exit 1; }
tail -2 gpurun_out/t3_tests.log
timeout -k 10 400 python -u benchmarks/attn_bench.py --chunks 576 > gpurun_out/t3_attn_bench.log 2>&1 || { tail -30 gpurun_out/t3_attn_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/t3_attn_bench.log
