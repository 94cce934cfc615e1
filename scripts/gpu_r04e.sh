#!/bin/bash
# Round 4 pass E: (1) kernel trace of the headline with --tool-frac 0.25 (where its extra step time goes),
# (2) HTTP TTFT with the Llama-3-class tokenizer, burst + staggered, (3) the 18k synthetic shared prefix through the API.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_tool25" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 --tool-frac 0.25 > "$R/gpurun_out/prof_tool25.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_tool25.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_tool25/run_kernel_trace.csv 60 > gpurun_out/shapes_tool25.txt 2>&1
head -30 gpurun_out/shapes_tool25.txt
bash scripts/gpu_r04c.sh
