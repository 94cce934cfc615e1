#!/bin/bash
# MFMA utilisation of tile attention v3 (attn_tile_kernel, variant 3): the engine's cascade pass (64 threads x 18k
# prefix keys, 576-key pieces) and planned causal prefills of 2k / 8k tokens. One PMC pass per case, kernel-trace
# only; summarised by scripts/pmc_mfma_summary.py into gpurun_out/pmc_tile3/summary.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_tile3
mkdir -p $OUT
for c in "3 576" "causal 2048 3" "causal 8192 3"; do
  tag=$(echo $c | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py $c > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/scripts/pmc_mfma_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
