#!/bin/bash
# Host-side cProfile of the headline bench vs --tool-frac 0.25, then a kernel trace of the headline by shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp; mkdir -p gpurun_out
for v in base tool25; do
  case $v in base) A="";; tool25) A="--tool-frac 0.25";; esac
  KAFKA_CPROFILE=$GRAFT_REPO_ROOT/gpurun_out/cprof_$v.txt timeout -k 10 300 python bench.py --steps 100 --warmup 20 $A > gpurun_out/cprof_bench_$v.log 2>&1 || { tail -20 gpurun_out/cprof_bench_$v.log; exit 1; }
  tail -1 gpurun_out/cprof_bench_$v.log | cut -c1-200
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_base" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 60 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof_base.log" 2>&1 || { tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof_base.log"; exit 1; }
cd "$GRAFT_REPO_ROOT" && python scripts/ktrace_shapes.py gpurun_out/prof_base/run_kernel_trace.csv 60 > gpurun_out/shapes_base.txt 2>&1
head -45 gpurun_out/shapes_base.txt
