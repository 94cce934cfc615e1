#!/bin/bash
# Round 4 pass I: early-launch overheads split: mode 3 = ordered launches without fences (atomics + polls only),
# mode 1 + poll back-off levels (any-order, no fences), mode 0 + back-off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for cfg in "KAFKA_EARLY=0" "KAFKA_EARLY=1 KAFKA_GATE_MODE=3" "KAFKA_EARLY=1 KAFKA_GATE_MODE=1 KAFKA_GATE_SLEEP=1" "KAFKA_EARLY=1 KAFKA_GATE_MODE=1 KAFKA_GATE_SLEEP=2" "KAFKA_EARLY=1 KAFKA_GATE_MODE=0 KAFKA_GATE_SLEEP=2"; do
  env $cfg timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_cfg.log 2>&1 || { tail -20 gpurun_out/bench_cfg.log; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/bench_cfg.log | cut -c1-150)"
done
