#!/bin/bash
# tile attention v3: numerics (attention tests) then the anatomy microbenchmark (+ ablations in $ABLS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn" --timeout 120 --timeout-method thread > gpurun_out/t3_tests.log 2>&1 || { tail -40 gpurun_out/t3_tests.log; exit 1; }
tail -2 gpurun_out/t3_tests.log
: > gpurun_out/anatomy.log
for abl in ${ABLS:-0}; do
  KAFKA_TILE_ABL=$abl timeout -k 10 300 python -u benchmarks/attn_tile_anatomy.py ${ANAT_ARGS:---variants 0,3 --keys 576,2304} 2>&1 | sed "s/^/abl$abl /" >> gpurun_out/anatomy.log || { tail -30 gpurun_out/anatomy.log; exit 1; }
done
grep keys_per gpurun_out/anatomy.log
