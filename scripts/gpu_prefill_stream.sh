#!/bin/bash
# Side-stream prefill attention (KAFKA_PREFILL_STREAM=1): engine GPU tests with it on, then the bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
KAFKA_PREFILL_STREAM=1 timeout -k 10 600 python -u -m pytest tests -m gpu -k "engine or smoke or prefix or cascade" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pstream.log 2>&1 || { tail -40 gpurun_out/t_pstream.log; exit 1; }
tail -2 gpurun_out/t_pstream.log
ARMS="KAFKA_PREFILL_STREAM=0;KAFKA_PREFILL_STREAM=1" ROUNDS=2 STEPS=200 WARM=20 bash scripts/gpu_ab_env.sh
