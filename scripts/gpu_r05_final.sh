#!/bin/bash
# Round-5 validation of the tree as committed: the whole GPU test suite, smoke(), bench 200/20 twice and the
# driver-shaped 20/5 (results under gpurun_out/final/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/final/pytest_gpu.log; [[ $rc == 0 ]] || { grep -E "FAILED|Error" gpurun_out/final/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
echo "smoke ok"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/final/bench_200_20_$i.log 2>&1 || { tail -20 gpurun_out/final/bench_200_20_$i.log; exit 1; }
  tail -1 gpurun_out/final/bench_200_20_$i.log | cut -c1-180
done
timeout -k 10 300 python bench.py > gpurun_out/final/bench_default.log 2>&1 || { tail -20 gpurun_out/final/bench_default.log; exit 1; }
tail -1 gpurun_out/final/bench_default.log | cut -c1-180
