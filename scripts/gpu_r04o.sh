#!/bin/bash
# Round 4 pass O: does the gate plumbing cost anything with gates off? Headline bench of the pre-gates commit
# (ab_old/, 3800543) vs this tree, interleaved x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
: > gpurun_out/bench_o.jsonl
for v in old new old new old new; do
  P=$R; [[ $v == old ]] && P=$R/ab_old
  (cd $P && PYTHONPATH=$P timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $R/gpurun_out/bench_$v.log 2>&1) || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/bench_o.jsonl
  echo "$v $(tail -1 gpurun_out/bench_$v.log | cut -c100-175)"
done
