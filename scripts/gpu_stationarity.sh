#!/bin/bash
# smoke (oracle-gap distribution) + the bench's short and long windows on one box: 20/5 at seeds 0..2 and 200/20
# at seed 0 (per-step log), so the stationarity of the headline bench can be read off one run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/stationarity.jsonl
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
for cfg in "20 5 0" "20 5 1" "20 5 2" "200 20 0" "200 20 1"; do
  set -- $cfg
  KAFKA_BENCH_STEPLOG=gpurun_out/steplog_$1_$2_s$3.jsonl timeout -k 10 300 python bench.py --steps $1 --warmup $2 \
    --seed $3 > gpurun_out/bench_$1_$2_s$3.log 2>&1 || { tail -20 gpurun_out/bench_$1_$2_s$3.log; exit 1; }
  tail -1 gpurun_out/bench_$1_$2_s$3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'steps': $1, 'warmup': $2, 'seed': $3, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'ttft_p50_ms': d.get('ttft_p50_ms')}))" | tee -a gpurun_out/stationarity.jsonl
done
