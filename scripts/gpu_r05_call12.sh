#!/bin/bash
# kernel trace of the headline with the split merge (decode partials + attn_merge_cascade)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sm" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_sm.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_sm.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_sm/run_kernel_trace.csv 60 > gpurun_out/shapes_sm.txt 2>&1; head -24 gpurun_out/shapes_sm.txt
