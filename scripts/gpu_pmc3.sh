#!/bin/bash
# PMC pass (own run, kernel-trace only): LDS pressure / stall counters of the cascade tile kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc3
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_ANY SQ_LDS_ADDR_CONFLICT -d $OUT/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
