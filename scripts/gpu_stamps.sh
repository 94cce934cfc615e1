#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT KAFKA_TILE_ABL=9
for nk in 576 2304; do timeout -k 10 120 python -u benchmarks/attn_tile_stamps.py $nk 2>&1 | grep -v amdgpu.ids; done
