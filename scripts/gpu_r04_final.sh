#!/bin/bash
# Round 4 final rehearsal: the full GPU test suite (one process, per-test timeouts), smoke(), bench 20/5 and 200/20,
# and a kernel trace of the headline by shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_gpu_full.log
[[ $rc == 0 ]] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu_full.log | head -20; tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20_5.log 2>&1 || { tail -20 gpurun_out/bench_20_5.log; exit 1; }
tail -1 gpurun_out/bench_20_5.log | cut -c1-220
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_200_20.log 2>&1 || { tail -20 gpurun_out/bench_200_20.log; exit 1; }
tail -1 gpurun_out/bench_200_20.log | cut -c1-220
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_final" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_final.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_final.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_final/run_kernel_trace.csv 60 > gpurun_out/shapes_final.txt 2>&1
head -3 gpurun_out/shapes_final.txt
