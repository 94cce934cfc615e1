#!/bin/bash
# one server, the burst load twice: does turn 0 of the SECOND burst still pay the first-burst TTFT (first-use costs)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
PORT=18631
KAFKA_LLM_BACKEND=engine KAFKA_MODEL=llama3-8b KAFKA_SANDBOX=none LOCAL_DB_PATH=:memory: KAFKA_IGNORE_EOS=1 \
  DEFAULT_MODEL=kafka timeout -k 10 500 python -m kafka_llm_service_amd.server --host 127.0.0.1 --port $PORT \
  > gpurun_out/serve_twice_server.log 2>&1 &
SRV=$!
ok=1
for i in 1 2 3; do
  timeout -k 10 300 python benchmarks/serve_bench.py --url http://127.0.0.1:$PORT --threads 64 --turns 4 \
    --max-tokens 128 > gpurun_out/serve_twice_$i.log 2>&1 || { ok=0; tail -20 gpurun_out/serve_twice_$i.log; break; }
  tail -1 gpurun_out/serve_twice_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($i, {k: d[k] for k in ('ttft_p50_ms','ttft_p99_ms','output_tok_s','ttft_p50_p99_ms_by_turn')})"
done
kill $SRV; wait $SRV
[[ $ok == 1 ]]
