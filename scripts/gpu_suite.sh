#!/bin/bash
# GPU validation of the tree as it is: the GPU test suite (once per SUITE_ENVS set, e.g. "base:KAFKA_X=0
# sc1:KAFKA_SC1_NORM=1,KAFKA_SC1_ROPE=1"), smoke(), and bench runs (BENCHES="200/20 200/20 20/5"). Output under
# gpurun_out/suite/. Stops at the first failure of the default set; later env sets only report.
# Usage: gpurun --timeout 1200 -- 'SUITE_ENVS="base:KAFKA_X=0" BENCHES="20/5" bash scripts/gpu_suite.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; O=gpurun_out/suite; mkdir -p $O
first=1
for set in ${SUITE_ENVS:-base:KAFKA_X=0}; do
  name=${set%%:*}; vars=${set#*:}
  env $(echo "$vars" | tr ',' ' ') timeout -k 10 1100 python -u -m pytest tests -m gpu -q -s --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS} > $O/pytest_$name.log 2>&1
  rc=$?; echo "== pytest $name: $(tail -1 $O/pytest_$name.log)"
  if [[ $rc != 0 ]]; then
    grep -E "^FAILED" $O/pytest_$name.log | head -20
    [[ $first == 1 ]] && exit 1
  fi
  first=0
done
if [[ -z $NO_SMOKE ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  grep -E "^smoke" $O/smoke.log | cut -c1-220
fi
i=0
for b in ${BENCHES}; do
  i=$((i + 1)); s=${b%/*}; w=${b#*/}
  timeout -k 10 300 python bench.py --steps $s --warmup $w ${BENCH_ARGS} > $O/bench_${s}_${w}_$i.log 2>&1 || { tail -20 $O/bench_${s}_${w}_$i.log; exit 1; }
  tail -1 $O/bench_${s}_${w}_$i.log | cut -c1-200
done
exit 0
