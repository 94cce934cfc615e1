#!/bin/bash
# Headline-bench A/B over environment settings, interleaved rounds in one box (cdna_hip_programming.md §5.4 rule 24).
# AB_SETS="name1:VAR=a,VAR2=b name2:VAR=c" AB_ROUNDS=2 AB_ARGS="--steps 200 --warmup 20"; one JSON line per run in
# gpurun_out/ab.jsonl (field "variant"). A name of the form name@dir runs bench.py from the tree `dir` (e.g. ab_prev:
# the previous commit's package with its own built .so) — code A/Bs in one box. Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
ARGS=${AB_ARGS:-"--steps 200 --warmup 20"}
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for set in $AB_SETS; do
    name=${set%%:*}; vars=${set#*:}; [[ "$vars" == "$set" ]] && vars=""
    tree=$GRAFT_REPO_ROOT
    if [[ "$name" == *@* ]]; then tree=$GRAFT_REPO_ROOT/${name#*@}; name=${name%%@*}; fi
    echo "== round $round $name ($vars) $(date +%T)"
    (cd $tree && env PYTHONPATH=$tree $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python bench.py $ARGS) \
      > gpurun_out/ab_$name.log 2>&1
    rc=$?
    if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/ab_$name.log; then echo "GPU fault in $name"; exit 3; fi
    [[ $rc == 0 ]] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/ab_$name.log; exit 1; }
    tail -1 gpurun_out/ab_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$name'; d['round']=$round; print(json.dumps(d))" >> gpurun_out/ab.jsonl
    tail -1 gpurun_out/ab.jsonl | cut -c1-200
  done
done
