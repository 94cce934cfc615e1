#!/bin/bash
# Round 4 pass AC: 33..64-row decode GEMMs as two XCD-shared 32-row tiles (KAFKA_WSTREAM_RT1=1: every CU streams,
# gate_up 448 workgroups instead of 224) — numerics under the switch, microbench at M = 64, bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_WSTREAM_RT1=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "wstream or engine_matches" > gpurun_out/t_ac.log 2>&1 || { tail -40 gpurun_out/t_ac.log; exit 1; }
tail -1 gpurun_out/t_ac.log
timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 64 --shapes 8b.gate_up,8b.qkv,8b.o,8b.down > gpurun_out/wsb_ac0.log 2>&1 || { tail -20 gpurun_out/wsb_ac0.log; exit 1; }
KAFKA_WSTREAM_RT1=1 timeout -k 10 200 python -u benchmarks/wstream_bench.py --M 64 --shapes 8b.gate_up,8b.qkv,8b.o,8b.down > gpurun_out/wsb_ac1.log 2>&1 || { tail -20 gpurun_out/wsb_ac1.log; exit 1; }
tail -4 gpurun_out/wsb_ac0.log; tail -4 gpurun_out/wsb_ac1.log
: > gpurun_out/bench_ac.jsonl
for round in 1 2; do
for cfg in "KAFKA_WSTREAM_RT1=0" "KAFKA_WSTREAM_RT1=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ac.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
