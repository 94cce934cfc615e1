#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of a short bench run, broken down by kernel and grid shape
# (scripts/ktrace_shapes.py: decode and mixed steps apart). KT_NAME names the output dir under gpurun_out/ktrace/,
# KT_ENV / KT_ARGS set the bench's environment / arguments. Counters go in their own run (scripts/gpu_pmc.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT; export KAFKA_NO_BUILD=1 TMPDIR=/tmp PYTHONPATH=$R; N=${KT_NAME:-default}; O=$R/gpurun_out/ktrace/$N
mkdir -p $O && cd /tmp
env ${KT_ENV:-KAFKA_X=0} timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O -o run --output-format csv -- \
  python3 $R/bench.py --steps ${KT_STEPS:-60} --warmup 20 ${KT_ARGS} > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
cd $R && python scripts/ktrace_shapes.py $O/run_kernel_trace.csv ${KT_STEPS:-60} > $O/shapes.txt 2>&1
python scripts/ktrace_gaps.py $O/run_kernel_trace.csv ${KT_STEPS:-60} > $O/gaps.txt 2>&1
# the raw trace (tens of MB) would push gpurun_out past what a call copies back: keep it only when asked
[[ -n $KT_KEEP_CSV ]] || rm -f $O/run_kernel_trace.csv
head -${KT_HEAD:-25} $O/shapes.txt
