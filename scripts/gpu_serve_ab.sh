#!/bin/bash
# HTTP burst A/B over environment settings on one box, interleaved rounds: AB_SETS="name:VAR=a,VAR2=b ..."
# one JSON line per run in gpurun_out/serve_ab.jsonl (fields arm, round, prompt)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/serve_ab.jsonl
for round in $(seq 1 ${AB_ROUNDS:-2}); do
  for prompt in ${PROMPTS:-reference}; do
    for set in $AB_SETS; do
      name=${set%%:*}; vars=${set#*:}; [[ "$vars" == "$set" ]] && vars=""
      echo "== round $round $prompt $name ($vars) $(date +%T)"
      env KAFKA_PROMPT=$prompt $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python benchmarks/serve_bench.py \
        --backend engine --model llama3-8b --threads 64 --turns 4 --max-tokens 128 $SERVE_EXTRA \
        > gpurun_out/serve_ab_$name.log 2>&1
      rc=$?
      if grep -q "HSA_STATUS_ERROR\|Memory access fault" gpurun_out/serve_ab_$name.log; then echo "GPU fault"; exit 3; fi
      [[ $rc == 0 ]] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/serve_ab_$name.log; exit 1; }
      tail -1 gpurun_out/serve_ab_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['arm']='$name'; d['round']=$round; d['prompt']='$prompt'; print(json.dumps(d))" >> gpurun_out/serve_ab.jsonl
      tail -1 gpurun_out/serve_ab.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('arm','prompt','ttft_p50_ms','ttft_p99_ms','output_tok_s')})"
    done
  done
done
