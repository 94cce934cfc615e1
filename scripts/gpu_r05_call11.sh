#!/bin/bash
# partials-only decode + attn_merge_cascade: numerics, then the cascade + decode pair timed both ways
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "merge or decode or cascade" > gpurun_out/call11_tests.log 2>&1 || { tail -30 gpurun_out/call11_tests.log; exit 1; }
tail -1 gpurun_out/call11_tests.log
timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_split2.jsonl 2>&1 || { tail -20 gpurun_out/cascade_split2.jsonl; exit 1; }
grep mode gpurun_out/cascade_split2.jsonl | cut -c1-75
