#!/bin/bash
# Round 5 baseline on this round's box: bench 200/20 twice, driver-shaped 20/5, and a kernel trace by shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/base_200_$i.log 2>&1 || { tail -20 gpurun_out/base_200_$i.log; exit 1; }
  tail -1 gpurun_out/base_200_$i.log | cut -c1-200
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/base_20_5.log 2>&1 || { tail -20 gpurun_out/base_20_5.log; exit 1; }
tail -1 gpurun_out/base_20_5.log | cut -c1-200
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_base" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_base.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_base.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_base/run_kernel_trace.csv 60 > gpurun_out/shapes_base.txt 2>&1
head -3 gpurun_out/shapes_base.txt
