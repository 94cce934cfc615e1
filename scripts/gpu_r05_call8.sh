#!/bin/bash
# fused-merge fp32 variant of the cascade bench + a fresh headline kernel trace (per-kernel time per step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_overlap4.jsonl 2>&1 || { tail -20 gpurun_out/cascade_overlap4.jsonl; exit 1; }
grep mode gpurun_out/cascade_overlap4.jsonl | cut -c1-60
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof/run_kernel_trace.csv 60 > gpurun_out/shapes.txt 2>&1; head -30 gpurun_out/shapes.txt
