#!/bin/bash
# PMC counters (own run, kernel-trace only) for the cascade tile kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py ${PMC_ARGS} > $OUT.log 2>&1 || { tail -20 $OUT.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py ${PMC_ARGS} >> $OUT.log 2>&1 || { tail -20 $OUT.log; exit 1; }
ls -R $OUT | head
