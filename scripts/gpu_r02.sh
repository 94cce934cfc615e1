#!/bin/bash
# Round-2 GPU session: GPU tests, smoke, headline bench at the driver's window (20/5) and a long window (200/20).
# Stops at the first failing step (no retries). Usage: gpurun --timeout 900 -- 'bash scripts/gpu_r02.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
fault() { if grep -q "HSA_STATUS_ERROR\|Memory access fault" "$1"; then echo "GPU fault in $1"; grep -m3 -B2 "HSA_STATUS_ERROR\|Memory access fault" "$1"; exit 3; fi; }
if [[ -z $SKIP_TESTS ]]; then
step tests
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${TEST_SEL} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; fault gpurun_out/pytest_gpu.log
[[ $rc == 0 ]] || { echo "tests failed rc=$rc"; grep -E "FAIL|ERROR" gpurun_out/pytest_gpu.log | tail -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; fault gpurun_out/smoke.log
[[ $rc == 0 ]] || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-300
fi
for W in ${WINDOWS:-20:5 200:20}; do
  K=${W%%:*}; WU=${W##*:}
  step "bench $K/$WU $BENCH_EXTRA"
  timeout -k 10 400 python bench.py --steps $K --warmup $WU $BENCH_EXTRA > gpurun_out/bench_${K}_${WU}.log 2>&1
  rc=$?; fault gpurun_out/bench_${K}_${WU}.log
  [[ $rc == 0 ]] || { echo "bench failed rc=$rc"; tail -30 gpurun_out/bench_${K}_${WU}.log; exit 1; }
  tail -1 gpurun_out/bench_${K}_${WU}.log
done
if [[ -n $PROF ]]; then
  step "rocprofv3 bench $PROF_ARGS"
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 80 --warmup 20 --ttft-samples 0 $PROF_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1)
  rc=$?; fault gpurun_out/prof.log
  [[ $rc == 0 ]] || { echo "prof failed rc=$rc"; tail -30 gpurun_out/prof.log; exit 1; }
  tail -1 gpurun_out/prof.log | cut -c1-200
  TR=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
  python scripts/ktrace_mix.py "$TR" 80 > gpurun_out/prof_breakdown.txt && cat gpurun_out/prof_breakdown.txt | head -70
  rm -f "$TR"
fi
echo "== done $(date +%T)"
