#!/bin/bash
# One gpurun call that collects every piece of single-GPU evidence, in order of importance; stops at the first
# failing step (no retries). Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_full.sh'
#   1. GPU test suite           -> gpurun_out/pytest_gpu.log
#   2. smoke()                  -> gpurun_out/smoke.log
#   3. headline bench (default) -> gpurun_out/bench.log
#   4. A/B: graphs / overlap    -> gpurun_out/ab.jsonl
#   5. MoE layer microbench     -> gpurun_out/moe_bench.log
#   6. rocprofv3 kernel stats   -> gpurun_out/prof/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { echo "== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-200
step bench
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
step ab
bash scripts/gpu_ab.sh || exit 1
step moe
timeout -k 10 300 python benchmarks/moe_bench.py > gpurun_out/moe_bench.log 2>&1 || { echo "moe bench failed"; tail -30 gpurun_out/moe_bench.log; exit 1; }
grep -v Warn gpurun_out/moe_bench.log
step prof
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 60 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1 || { echo "prof failed"; tail -30 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"; exit 1; }
tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof.log" | cut -c1-200
echo "== done $(date +%T)"
