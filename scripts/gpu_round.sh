#!/bin/bash
# One GPU-box session: kernel/engine GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats of a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp
mkdir -p gpurun_out
STEP=${1:-all}
if [[ $STEP == all || $STEP == test ]]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -40 gpurun_out/smoke.log; exit 1; }
  tail -2 gpurun_out/smoke.log
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
if [[ $STEP == all || $STEP == prof ]]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 60 --warmup 20 ${PROF_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "prof failed"; tail -40 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
  tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
  find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head -5
fi
