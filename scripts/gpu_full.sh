#!/bin/bash
# One gpurun call that collects every piece of single-GPU evidence, in order of importance; stops at the first
# failing step (no retries) and at the first GPU runtime fault printed by any step.
# Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_full.sh'
#   1. GPU test suite                      -> gpurun_out/pytest_gpu.log
#   2. smoke()                             -> gpurun_out/smoke.log
#   3. headline bench A/B + rocprofv3 stats -> gpurun_out/ab.jsonl, gpurun_out/prof/  (scripts/gpu_bench_ab.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
fault() { if grep -q "HSA_STATUS_ERROR\|Memory access fault" "$1"; then echo "GPU fault in $1"; grep -m3 -B2 "HSA_STATUS_ERROR\|Memory access fault" "$1"; exit 3; fi; }
step tests
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; fault gpurun_out/pytest_gpu.log
[[ $rc == 0 ]] || { echo "tests failed rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_gpu.log | tail -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
[[ -n $SKIP_SMOKE ]] || {
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; fault gpurun_out/smoke.log
[[ $rc == 0 ]] || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
}
[[ -n $SKIP_BENCH ]] || bash scripts/gpu_bench_ab.sh || exit 1
echo "== done $(date +%T)"
