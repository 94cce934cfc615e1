#!/bin/bash
# Round-end rehearsal (scripts/gpu_final.sh) + a kernel trace of a short bench broken down by kernel and grid shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/gpu_final.sh || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_final" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 60 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_final.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_final.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python scripts/ktrace_shapes.py gpurun_out/prof_final/run_kernel_trace.csv 60 > gpurun_out/shapes_final.txt 2>&1
head -30 gpurun_out/shapes_final.txt
