#!/bin/bash
# Decode attention on the headline shape: timing sweep (benchmarks/decode_bench.py) + per-layout PMC passes
# (HBM bytes, L2 hit rate, wave waits). Usage: gpurun -- 'bash scripts/gpu_r05_decode_pmc.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT; mkdir -p gpurun_out/dpmc
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python benchmarks/decode_bench.py --targets ${DB_TARGETS:-768,1344,2048} > gpurun_out/dpmc/sweep.jsonl 2>&1 || { tail -20 gpurun_out/dpmc/sweep.jsonl; exit 1; }
cat gpurun_out/dpmc/sweep.jsonl
cd /tmp
for lay in contiguous scattered; do
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d "$R/gpurun_out/dpmc/${lay}_${tag}" -o run --output-format csv -- python3 "$R/benchmarks/decode_bench.py" --layouts $lay --plans adaptive --layers 4 > "$R/gpurun_out/dpmc/${lay}_${tag}.log" 2>&1 || { echo "pmc $lay $tag failed"; tail -5 "$R/gpurun_out/dpmc/${lay}_${tag}.log"; exit 1; }
  done
done
cd "$R" && for d in gpurun_out/dpmc/*/; do echo "## $d"; python scripts/pmc_kernels.py "$d" attn_decode; done > gpurun_out/dpmc/summary.txt 2>&1; cat gpurun_out/dpmc/summary.txt
