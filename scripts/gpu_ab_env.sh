#!/bin/bash
# A/B of bench.py under different environment settings, one box, interleaved rounds.
# An arm may name AB_DIR=<subdir>: a second tree (e.g. `git archive` of an older commit, built in place) to
# bench from instead of the repo root; FLAG=--x passes a bench.py flag to that arm only.
# Usage: gpurun -- 'ARMS="A=1;A=2" ROUNDS=2 STEPS=60 WARM=20 bash scripts/gpu_ab_env.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
IFS=';' read -ra arms <<< "$ARMS"
for r in $(seq 1 ${ROUNDS:-2}); do
  for a in "${arms[@]}"; do
    echo "== round $r arm [$a] $(date +%T)"
    dir=$GRAFT_REPO_ROOT
    flags=""
    for kv in $a; do [[ $kv == AB_DIR=* ]] && dir=$GRAFT_REPO_ROOT/${kv#AB_DIR=}; [[ $kv == FLAG=* ]] && flags="$flags ${kv#FLAG=}"; done
    (cd $dir && env $a PYTHONPATH=$dir timeout -k 10 300 python bench.py --steps ${STEPS:-60} --warmup ${WARM:-20} $BENCH_EXTRA $flags) > gpurun_out/ab.log 2>&1
    rc=$?
    if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/ab.log; then echo "GPU fault"; tail -20 gpurun_out/ab.log; exit 3; fi
    [[ $rc == 0 ]] || { echo "bench failed rc=$rc"; tail -30 gpurun_out/ab.log; exit 1; }
    tail -1 gpurun_out/ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'arm': '$a', 'round': $r, 'tok_s': d['value'], 'ms': d['ms_per_step'], 'ttft': d['ttft_p50_ms']}))" | tee -a gpurun_out/ab.jsonl
  done
done
if [[ -n $CPROF ]]; then
  echo "== cprofile $(date +%T)"
  env $CPROF KAFKA_CPROFILE=gpurun_out/cprof.txt timeout -k 10 300 python bench.py --steps 60 --warmup 20 --ttft-samples 0 > gpurun_out/cprof_run.log 2>&1 || { tail -20 gpurun_out/cprof_run.log; exit 1; }
  head -70 gpurun_out/cprof.txt
fi
