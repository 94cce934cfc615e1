#!/bin/bash
# round 3: kernels + engine + custom all-reduce GPU tests, then the attention microbenchmark
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_custom_allreduce_gpu.py -x -v --timeout 280 --timeout-method thread > gpurun_out/r03a_tests.log 2>&1 || { tail -40 gpurun_out/r03a_tests.log; exit 1; }
tail -3 gpurun_out/r03a_tests.log
timeout -k 10 400 python -u benchmarks/attn_bench.py --chunks 576 > gpurun_out/r03a_attn_bench.log 2>&1 || { tail -30 gpurun_out/r03a_attn_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03a_attn_bench.log
