#!/bin/bash
# Round 4 pass H: where early-launched layers lose time. Engine equality test (2-chunk weight prefetch), then bench
# EARLY=0 vs EARLY=1 with gate modes: 0 = full release/acquire, 1 = no fences (timing only), 2 = ordered launches
# (barrier bit kept, gates still waited on); a kernel trace of EARLY=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "early" > gpurun_out/t_early.log 2>&1 || { tail -60 gpurun_out/t_early.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_early.log | tail -2
for cfg in "KAFKA_EARLY=0" "KAFKA_EARLY=1 KAFKA_GATE_MODE=0" "KAFKA_EARLY=1 KAFKA_GATE_MODE=1" "KAFKA_EARLY=1 KAFKA_GATE_MODE=2"; do
  env $cfg timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c1-150)"
done
cd /tmp && KAFKA_EARLY=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_early" -o run --output-format csv -- python3 "$R/bench.py" --steps 30 --warmup 10 > "$R/gpurun_out/prof_early.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_early.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_early/run_kernel_trace.csv 30 > gpurun_out/shapes_early.txt 2>&1
head -30 gpurun_out/shapes_early.txt
