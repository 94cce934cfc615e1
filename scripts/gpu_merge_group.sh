#!/bin/bash
# Decode fused-merge load group size: kernel tests at 16 and 32, then the bench A/B 8 / 16 / 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
for g in 16 32; do
KAFKA_DECODE_MERGE_GROUP=$g timeout -k 10 300 python -u -m pytest tests -m gpu -k "decode or cascade or engine" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mg$g.log 2>&1 || { tail -40 gpurun_out/t_mg$g.log; exit 1; }
tail -1 gpurun_out/t_mg$g.log
done
ARMS="KAFKA_DECODE_MERGE_GROUP=8;KAFKA_DECODE_MERGE_GROUP=16;KAFKA_DECODE_MERGE_GROUP=32" ROUNDS=2 STEPS=200 WARM=20 bash scripts/gpu_ab_env.sh
