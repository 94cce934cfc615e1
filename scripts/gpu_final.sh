#!/bin/bash
# Round-end rehearsal: GPU suite, smoke(), default bench (20/5 and 200/20) — what the driver runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20_5.log 2>&1 || { tail -20 gpurun_out/bench_20_5.log; exit 1; }
tail -1 gpurun_out/bench_20_5.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_200_20.log 2>&1 || { tail -20 gpurun_out/bench_200_20.log; exit 1; }
tail -1 gpurun_out/bench_200_20.log
