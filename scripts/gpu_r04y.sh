#!/bin/bash
# Round 4 pass Y: hipBLASLt orientation for mixed-step projections (x W^T vs W x^T).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u benchmarks/blas_orient_bench.py > gpurun_out/blas_orient.jsonl 2> gpurun_out/blas_orient.err || { tail -20 gpurun_out/blas_orient.err; exit 1; }
cat gpurun_out/blas_orient.jsonl
