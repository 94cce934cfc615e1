#!/bin/bash
# Cascade shape (benchmarks/attn_one.py 3 576): where the tile loop's cycles go — LDS issue / bank conflicts, VALU,
# MFMA, waits, TA. One counter pass per run (kernel-trace only), each under its own kill timeout.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/tpmc
mkdir -p $OUT
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_BUSY_max TD_BUSY_avr TD_BUSY_max GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py 3 576 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -8 $OUT/p$i.log; break; }
done
cd $GRAFT_REPO_ROOT && for d in gpurun_out/tpmc/p*/; do echo "## $d"; python scripts/pmc_kernels.py "$d" attn_tile; done > gpurun_out/tpmc/summary.txt 2>&1; cat gpurun_out/tpmc/summary.txt
