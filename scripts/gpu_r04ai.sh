#!/bin/bash
# Round 4 pass AI: two K halves per chunk (8 waves) for the long 64-row decode streams (KAFKA_WSTREAM_KW2=1:
# gate_up unsplit with its fused SwiGLU, down) — numerics under the switch, then bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_WSTREAM_KW2=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream or engine_matches" > gpurun_out/t_ai.log 2>&1 || { tail -40 gpurun_out/t_ai.log; exit 1; }
tail -1 gpurun_out/t_ai.log
: > gpurun_out/bench_ai.jsonl
for round in 1 2 3; do
for cfg in "KAFKA_WSTREAM_KW2=0" "KAFKA_WSTREAM_KW2=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ai.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
