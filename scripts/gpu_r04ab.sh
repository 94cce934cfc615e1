#!/bin/bash
# Round 4 pass AB: fused QKV + RoPE epilogue with batched position / cos-sin / slot loads — numerics, bench A/B
# against the separate rope_kv launch, and a trace of the fused kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "qkv_rope" > gpurun_out/t_ab.log 2>&1 || { tail -40 gpurun_out/t_ab.log; exit 1; }
KAFKA_FUSE_QKV_ROPE=1 timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "engine_matches or cascade" >> gpurun_out/t_ab.log 2>&1 || { tail -40 gpurun_out/t_ab.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_ab.log
: > gpurun_out/bench_ab.jsonl
for round in 1 2; do
for cfg in "KAFKA_FUSE_QKV_ROPE=0" "KAFKA_FUSE_QKV_ROPE=1"; do
  env $cfg timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  tail -1 gpurun_out/bench_cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$cfg'; print(json.dumps(d))" >> gpurun_out/bench_ab.jsonl
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c60-140)"
done
done
export KAFKA_FUSE_QKV_ROPE=1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fuse2" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_fuse2.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_fuse2.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_fuse2/run_kernel_trace.csv 60 > gpurun_out/shapes_fuse2.txt 2>&1
grep -E "== decode|tru grid" gpurun_out/shapes_fuse2.txt | head -6
