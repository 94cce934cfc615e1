#!/bin/bash
# MFMA utilisation of the tile attention kernel (one PMC pass, kernel-trace only): cascade pass and planned causal
# prefills. Summarised by scripts/pmc_mfma_summary.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_mfma
mkdir -p $OUT
for c in "0 576" "causal 2048" "causal 8192"; do
  tag=$(echo $c | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/$tag -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py $c > $OUT/$tag.log 2>&1 || { tail -20 $OUT/$tag.log; exit 1; }
done
ls -R $OUT | head -30
