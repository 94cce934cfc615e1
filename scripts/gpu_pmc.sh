#!/bin/bash
# PMC counters, one pass per counter group (rocprofv3 does not split passes; each run kernel-trace only, never with a
# system / runtime trace), over PMC_CMD (a python script + args under the repo, default the cascade tile shape).
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp KAFKA_NO_BUILD=1 PYTHONPATH=$R; O=$R/gpurun_out/pmc/${PMC_NAME:-run}; mkdir -p $O
cd /tmp
CMD=${PMC_CMD:-benchmarks/attn_one.py 3 576}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           ${PMC_EXTRA}; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $O/p$i -o p$i --output-format csv -- python3 $R/$CMD >> $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
done
ls -R $O | head
