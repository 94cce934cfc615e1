#!/bin/bash
# PMC passes (each its own run, kernel-trace only) for the cascade tile kernel: instruction mix and pipe occupancy.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc2
mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS -d $OUT/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py > $OUT/p1.log 2>&1 || { tail -20 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_one.py > $OUT/p2.log 2>&1 || { tail -20 $OUT/p2.log; exit 1; }
find $OUT -name "*counter_collection.csv" | head
