#!/bin/bash
# Round 4 pass AA: kernel trace of the headline with the fused QKV + RoPE epilogue (KAFKA_FUSE_QKV_ROPE=1) — where
# its measured -5 % comes from.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export KAFKA_FUSE_QKV_ROPE=1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fuse" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_fuse.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_fuse.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_fuse/run_kernel_trace.csv 60 > gpurun_out/shapes_fuse.txt 2>&1
head -24 gpurun_out/shapes_fuse.txt
