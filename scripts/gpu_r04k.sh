#!/bin/bash
# Round 4 pass K: the full GPU test suite (one process, per-test timeouts), smoke(), bench 20/5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_gpu_full.log | tail -5
[[ $rc == 0 ]] || { grep -E "FAILED|Error|error" gpurun_out/pytest_gpu_full.log | head -20; tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_20_5.log 2>&1 || { tail -20 gpurun_out/bench_20_5.log; exit 1; }
tail -1 gpurun_out/bench_20_5.log | cut -c1-200
