#!/bin/bash
# Weight-streaming decode GEMM evidence, part 1: its kernel tests, its microbench vs hipBLASLt, the GPU suite, smoke.
# Stops at the first failing step (no retries). Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_stream.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
step wstream-tests
timeout -k 10 400 $PT tests/test_kernels_gpu.py -k "wstream or slab" > gpurun_out/pytest_ws.log 2>&1 || { echo "wstream tests failed"; tail -40 gpurun_out/pytest_ws.log; exit 1; }
tail -2 gpurun_out/pytest_ws.log
step wstream-bench
timeout -k 10 300 python benchmarks/wstream_bench.py > gpurun_out/wstream_bench.log 2>&1 || { echo "wstream bench failed"; tail -30 gpurun_out/wstream_bench.log; exit 1; }
grep -v Warn gpurun_out/wstream_bench.log | cut -c1-300
step gpu-tests
timeout -k 10 900 $PT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
echo "== done $(date +%T)"
