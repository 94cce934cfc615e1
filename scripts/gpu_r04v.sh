#!/bin/bash
# Round 4 pass V: row tiles on one XCD (64-row tiles sharing each weight slice in L2, KAFKA_WSTREAM_ROWSPLIT=1) —
# kernel tests (default + switch), then bench A/B: default, rowsplit, rowsplit with 129..256-row steps streamed too.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream" > gpurun_out/t_v.log 2>&1 || { tail -40 gpurun_out/t_v.log; exit 1; }
tail -1 gpurun_out/t_v.log
KAFKA_WSTREAM_ROWSPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream or engine_matches or cascade" > gpurun_out/t_v2.log 2>&1 || { tail -40 gpurun_out/t_v2.log; exit 1; }
echo "rowsplit: $(tail -1 gpurun_out/t_v2.log)"
timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 100 > gpurun_out/wsb_default.log 2>&1 || true
KAFKA_WSTREAM_ROWSPLIT=1 timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 100 > gpurun_out/wsb_rowsplit.log 2>&1 || true
tail -6 gpurun_out/wsb_default.log; tail -6 gpurun_out/wsb_rowsplit.log
: > gpurun_out/bench_v.jsonl
for round in 1 2; do
for cfg in "KAFKA_WSTREAM_ROWSPLIT=0" "KAFKA_WSTREAM_ROWSPLIT=1" "KAFKA_WSTREAM_ROWSPLIT=1 KAFKA_STREAM_MAX_M=256"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_v.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c100-175)"
done
done
tail -1 gpurun_out/bench_v.jsonl | python -c "import json,sys; print(json.loads(sys.stdin.read())['step_rows_hist'])"
