#!/bin/bash
# cascade prefix pass: sequential vs concurrent with the suffix decode kernel (two streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_overlap.jsonl 2>&1 || { tail -20 gpurun_out/cascade_overlap.jsonl; exit 1; }
cat gpurun_out/cascade_overlap.jsonl
timeout -k 10 300 python benchmarks/moe_bench.py 1,16,64,128,256 > gpurun_out/moe_pin.jsonl 2>&1 || { tail -20 gpurun_out/moe_pin.jsonl; exit 1; }
cat gpurun_out/moe_pin.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "grouped or moe" > gpurun_out/call5_tests.log 2>&1 || { tail -30 gpurun_out/call5_tests.log; exit 1; }
tail -1 gpurun_out/call5_tests.log
