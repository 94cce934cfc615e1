#!/bin/bash
# Llama-3-70B on one GPU (tiled-only weights): row fit at the streaming kernel's 256-row limit (default), at 128, off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
ARMS="X=0;KAFKA_STEP_ROWS_FIT=128" ROUNDS=1 STEPS=60 WARM=10 BENCH_EXTRA="--model llama3-70b --threads 64" bash scripts/gpu_ab_env.sh
