#!/bin/bash
# Same-box interleaved headline A/B: the working tree (new) against the snapshot in ab_old/ (old), then the GPU
# kernel tests of the new tree. Usage: gpurun -- 'AB_PAIRS=3 bash scripts/gpu_r05_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export KAFKA_NO_BUILD=1 TMPDIR=/tmp; mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
ARGS=${AB_ARGS:-"--steps 200 --warmup 20"}
: > gpurun_out/ab.jsonl
run() {  # name dir
  ( cd "$2" && PYTHONPATH="$2" timeout -k 10 300 python bench.py $ARGS > "$R/gpurun_out/ab_$1.log" 2>&1 ) || { echo "$1 failed"; tail -20 "gpurun_out/ab_$1.log"; exit 1; }
  tail -1 "gpurun_out/ab_$1.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); d['variant']='$1'; print(json.dumps(d))" >> gpurun_out/ab.jsonl
  tail -1 gpurun_out/ab.jsonl | cut -c1-160
}
# variants: new (this tree), old (ab_old/), prev (ab_prev/: the last commit, built), newg (this tree, --graphs),
# newe (this tree + $AB_ENV env)
for i in $(seq 1 ${AB_PAIRS:-2}); do
  for v in ${AB_SEQ:-new old}; do
    case $v in
      new) run new$i "$R" ;;
      old) run old$i "$R/ab_old" ;;
      prev) run prev$i "$R/ab_prev" ;;
      newg) ARGS="$ARGS --graphs" run newg$i "$R" ;;
      newe) env $AB_ENV bash -c true && ( export $AB_ENV; run newe$i "$R" ) || exit 1 ;;
    esac
  done
done
if [[ -n $AB_DECODE ]]; then
  PYTHONPATH=$R timeout -k 10 300 python benchmarks/decode_bench.py $AB_DECODE > gpurun_out/decode_bench.log 2>&1 || { tail -20 gpurun_out/decode_bench.log; exit 1; }
  cat gpurun_out/decode_bench.log
fi
if [[ -n $AB_TESTS ]]; then
  PYTHONPATH=$R timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $AB_TESTS > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [[ $rc == 0 ]] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit 1; }
fi
if [[ -n $AB_PROF ]]; then
  cd /tmp && PYTHONPATH=$R timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 60 --warmup 20 > "$R/gpurun_out/prof.log" 2>&1 || { tail -30 "$R/gpurun_out/prof.log"; exit 1; }
  cd "$R" && python scripts/ktrace_shapes.py gpurun_out/prof/run_kernel_trace.csv 60 > gpurun_out/shapes.txt 2>&1; head -3 gpurun_out/shapes.txt
fi
