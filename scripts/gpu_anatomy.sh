#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
: > gpurun_out/anatomy.log
for abl in ${ABLS:-0 1 2 3}; do
  KAFKA_TILE_ABL=$abl timeout -k 10 300 python -u benchmarks/attn_tile_anatomy.py --variants 3 --keys 576,2304 ${ANAT_ARGS} 2>&1 | sed "s/^/abl$abl /" >> gpurun_out/anatomy.log || { tail -30 gpurun_out/anatomy.log; exit 1; }
done
grep keys_per gpurun_out/anatomy.log
