#!/bin/bash
# merge variants of the cascade + suffix decode, then config 4 at real size (Llama-3-70B agent run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/cascade_overlap_bench.py > gpurun_out/cascade_overlap3.jsonl 2>&1 || { tail -20 gpurun_out/cascade_overlap3.jsonl; exit 1; }
grep mode gpurun_out/cascade_overlap3.jsonl
SKIP_MIXTRAL=1 bash scripts/gpu_r05_configs.sh
