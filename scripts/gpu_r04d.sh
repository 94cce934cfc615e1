#!/bin/bash
# Round 4 pass D: (1) attention kernel tests on the new build, (2) tile-kernel anatomy + headline bench A/B of the
# previous commit's build (ab_old/) vs this tree, interleaved, (3) host cProfile of the headline and --tool-frac 0.25,
# (4) a kernel trace of the headline by shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
PYTHONPATH=$R timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn" --timeout 120 --timeout-method thread > gpurun_out/t_attn.log 2>&1 || { tail -40 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
: > gpurun_out/anat_ab.log
for v in old new old new; do
  P=$R; [[ $v == old ]] && P=$R/ab_old
  PYTHONPATH=$P timeout -k 10 200 python -u benchmarks/attn_tile_anatomy.py --variants 3 --keys 576,2304 2>&1 | grep keys_per | sed "s/^/$v /" >> gpurun_out/anat_ab.log || { echo "anatomy $v failed"; exit 1; }
done
cat gpurun_out/anat_ab.log
: > gpurun_out/bench_old_new.jsonl
for v in old new old new; do
  P=$R; [[ $v == old ]] && P=$R/ab_old
  (cd $P && PYTHONPATH=$P timeout -k 10 300 python bench.py --steps 200 --warmup 20 > $R/gpurun_out/bench_$v.log 2>&1) || { tail -20 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$v'; print(json.dumps(d))" >> gpurun_out/bench_old_new.jsonl
  tail -1 gpurun_out/bench_old_new.jsonl | cut -c1-160
done
export PYTHONPATH=$R
for v in base tool25; do
  case $v in base) A="";; tool25) A="--tool-frac 0.25";; esac
  KAFKA_CPROFILE=$R/gpurun_out/cprof_$v.txt timeout -k 10 300 python bench.py --steps 100 --warmup 20 $A > gpurun_out/cprof_bench_$v.log 2>&1 || { tail -20 gpurun_out/cprof_bench_$v.log; exit 1; }
  tail -1 gpurun_out/cprof_bench_$v.log | cut -c1-200
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_base" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof_base.log" 2>&1 || { tail -30 "$R/gpurun_out/prof_base.log"; exit 1; }
cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof_base/run_kernel_trace.csv 60 > gpurun_out/shapes_base.txt 2>&1
head -60 gpurun_out/shapes_base.txt
