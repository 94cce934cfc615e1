#!/bin/bash
# Round 4 pass U: four row tiles on 256-deep chunks (97..128-row steps) — kernel tests under the switch, then a bench
# A/B vs the 128-deep default (the report's step_rows_hist shows how many steps each plan covers).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_WSTREAM_MT4_KC=256 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream" > gpurun_out/t_u.log 2>&1 || { tail -40 gpurun_out/t_u.log; exit 1; }
tail -1 gpurun_out/t_u.log
: > gpurun_out/bench_u.jsonl
for round in 1 2 3; do
for cfg in "KAFKA_WSTREAM_MT4_KC=128" "KAFKA_WSTREAM_MT4_KC=256"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_u.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c100-175)"
done
done
tail -1 gpurun_out/bench_u.jsonl | python -c "import json,sys; print(json.loads(sys.stdin.read())['step_rows_hist'])"
