#!/bin/bash
# Llama-3-70B on one GPU (tiled-only weights): row fit on (default in tiled-only mode) vs off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
ARMS="X=0;KAFKA_STEP_ROWS_FIT=0" ROUNDS=1 STEPS=60 WARM=10 BENCH_EXTRA="--model llama3-70b --threads 64" bash scripts/gpu_ab_env.sh
