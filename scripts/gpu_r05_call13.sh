#!/bin/bash
# one-round-trip attn_merge_cascade: numerics, headline A/B against the last commit (fused ticket merge), trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "merge or decode or cascade" > gpurun_out/call13_tests.log 2>&1 || { tail -30 gpurun_out/call13_tests.log; exit 1; }
tail -1 gpurun_out/call13_tests.log
AB_PAIRS=3 AB_SEQ="new prev" bash scripts/gpu_r05_ab.sh || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sm2" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_sm2.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_sm2.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_sm2/run_kernel_trace.csv 60 > gpurun_out/shapes_sm2.txt 2>&1; grep -E "decode:|merge_cascade|attn_decode_kernel<128, false>  .*grid \(2048, 194" gpurun_out/shapes_sm2.txt
