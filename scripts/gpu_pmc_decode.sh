#!/bin/bash
# PMC passes (kernel-trace only, one counter group per run) over the engine's cascade + suffix decode pair on the
# bench's suffix-length law (benchmarks/attn_partition_bench.py --seq-only): wave occupancy / wait / busy and bytes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_decode
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/benchmarks/attn_partition_bench.py --seq-only > $OUT/p$i.log 2>&1 || { tail -20 $OUT/p$i.log; exit 1; }
done
ls -R $OUT | head -30
